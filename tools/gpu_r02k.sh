#!/bin/bash
# Grid batches assembling bodies on the tail: full GPU suite, config 1 line.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02k
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/all.log 2>&1 || { echo ALL_FAILED; tail -30 $OUT/all.log; exit 1; }
tail -1 $OUT/all.log
timeout -k 10 300 python -u bench.py --config 1 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c1.log 2>&1 || { echo C1_FAILED; tail -20 $OUT/c1.log; exit 1; }
echo "c1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/c1.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/c1.log)"
