#!/bin/bash
# Speculated-producer lead of 4 and 6 KiB against the default 12 KiB: unique
# tests, config 2 step time and k_data_blocks FETCH_SIZE (varlib/ builds).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02zk
mkdir -p $OUT
for v in default l4 l6; do
if [ $v = default ]; then unset TBC_LIB; else export TBC_LIB=$PWD/varlib/libtbc_$v.so; fi
timeout -k 10 200 python -u -m pytest tests/test_gpu_unique.py -x -q --timeout 150 --timeout-method thread > $OUT/tests_$v.log 2>&1 || { echo TESTS_${v}_FAILED; tail -30 $OUT/tests_$v.log; exit 1; }
timeout -k 10 200 python -u bench.py --config 2 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c2_$v.log 2>&1 || { echo C2_${v}_FAILED; tail -20 $OUT/c2_$v.log; exit 1; }
echo "$v $(tail -1 $OUT/tests_$v.log) $(grep -o '"ms_per_step": [0-9.]*' $OUT/c2_$v.log) $(grep -o '"data_blocks": [0-9.]*' $OUT/c2_$v.log)"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$v -o run -- python3 -u bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/fetch_$v.log 2>&1 || { echo FETCH_${v}_FAILED; tail -20 $OUT/fetch_$v.log; exit 1; }
done
echo ALL_OK
