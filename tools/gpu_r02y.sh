#!/bin/bash
# Config 5: groups x col2.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02y
mkdir -p $OUT
TBC_COL2_MIN_WAVES=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_col2.py -x -q --timeout 200 --timeout-method thread > $OUT/col2.log 2>&1 || { echo COL2_FAILED; tail -40 $OUT/col2.log; exit 1; }
tail -1 $OUT/col2.log
for g in 1 2; do
TBC_GROUPS=$g timeout -k 10 200 python -u bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/c5_g$g.log 2>&1 || { echo C5_FAILED; tail -20 $OUT/c5_g$g.log; exit 1; }
echo "g=$g col2 $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5_g$g.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/c5_g$g.log)"
done
timeout -k 10 200 python -u bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/c5.log 2>&1 || { echo C5D_FAILED; tail -20 $OUT/c5.log; exit 1; }
echo "default $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5.log)"
