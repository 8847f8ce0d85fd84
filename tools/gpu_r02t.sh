#!/bin/bash
# Full GPU suite, then bench lines of configs 1-5 with the current lib.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02t
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/all.log 2>&1 || { echo ALL_FAILED; tail -30 $OUT/all.log; exit 1; }
tail -1 $OUT/all.log
for c in 2 3 4 5; do
timeout -k 10 240 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c$c.log 2>&1 || { echo C${c}_FAILED; tail -20 $OUT/c$c.log; exit 1; }
echo "c$c $(grep -o '"ms_per_step": [0-9.]*' $OUT/c$c.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/c$c.log)"
done
timeout -k 10 400 python -u bench.py --config 1 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c1.log 2>&1 || { echo C1_FAILED; tail -20 $OUT/c1.log; exit 1; }
echo "c1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/c1.log)"
