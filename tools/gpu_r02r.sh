#!/bin/bash
# Producer timing split (spec_probe) for configs 2 and 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02r
mkdir -p $OUT
TBC_PROBE_PRODUCERS_ONLY=1 timeout -k 10 200 python -u tools/spec_probe.py --config 2 --jobs 8 > $OUT/p2.json 2>&1 || { echo P2_FAILED; tail -20 $OUT/p2.json; exit 1; }
cat $OUT/p2.json
TBC_PROBE_PRODUCERS_ONLY=1 timeout -k 10 200 python -u tools/spec_probe.py --config 4 --jobs 10 > $OUT/p4.json 2>&1 || { echo P4_FAILED; tail -20 $OUT/p4.json; exit 1; }
cat $OUT/p4.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_unique.py -x -q --timeout 120 --timeout-method thread > $OUT/unique.log 2>&1 || { echo UNIQUE_FAILED; tail -30 $OUT/unique.log; exit 1; }
tail -1 $OUT/unique.log
for c in 2 4; do
timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c$c.log 2>&1 || { echo C${c}_FAILED; tail -20 $OUT/c$c.log; exit 1; }
echo "c$c $(grep -o '"ms_per_step": [0-9.]*' $OUT/c$c.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/c$c.log)"
done
