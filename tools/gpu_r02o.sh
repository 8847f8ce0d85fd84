#!/bin/bash
# Speculation: tests, full lines of configs 2 and 4, then the producer-only timing probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02o
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_unique.py -x -q --timeout 120 --timeout-method thread > $OUT/unique.log 2>&1 || { echo UNIQUE_FAILED; tail -30 $OUT/unique.log; exit 1; }
tail -1 $OUT/unique.log
for c in 2 4; do
timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c$c.log 2>&1 || { echo C${c}_FAILED; tail -20 $OUT/c$c.log; exit 1; }
echo "c$c $(grep -o '"ms_per_step": [0-9.]*' $OUT/c$c.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/c$c.log)"
done
for c in 2 4; do
TBC_PROBE_PRODUCERS_ONLY=1 timeout -k 10 200 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $OUT/p$c.log 2>&1 || { echo P${c}_FAILED; tail -20 $OUT/p$c.log; exit 1; }
echo "p$c $(grep -o '"ms_per_step": [0-9.]*' $OUT/p$c.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/p$c.log)"
TBC_PROBE_PRODUCERS_ONLY=1 TBC_NO_SPECULATION=1 timeout -k 10 200 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $OUT/pn$c.log 2>&1 || { echo PN${c}_FAILED; tail -20 $OUT/pn$c.log; exit 1; }
echo "pn$c $(grep -o '"ms_per_step": [0-9.]*' $OUT/pn$c.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/pn$c.log)"
done
