#!/bin/bash
# Producer throttle (speculated producers stay <= 12 KiB ahead of their chain):
# unique + parity tests, configs 2 and 4, a FETCH_SIZE pass on config 2.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02z
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_unique.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in 2 4; do
timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c$c.log 2>&1 || { echo C${c}_FAILED; tail -20 $OUT/c$c.log; exit 1; }
echo "c$c $(grep -o '"ms_per_step": [0-9.]*' $OUT/c$c.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/c$c.log)"
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 -u bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/fetch.log 2>&1 || { echo FETCH_FAILED; tail -20 $OUT/fetch.log; exit 1; }
echo FETCH_OK
