#!/bin/bash
# Config 5: job-group size ratio sweep (and group count).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02w
mkdir -p $OUT
for r in 1.0 0.8 0.65 0.5; do
TBC_GROUP_RATIO=$r timeout -k 10 200 python -u bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/c5_$r.log 2>&1 || { echo C5_FAILED; tail -20 $OUT/c5_$r.log; exit 1; }
echo "r=$r $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5_$r.log)"
done
for g in 5 6; do
TBC_GROUPS=$g TBC_GROUP_RATIO=0.65 timeout -k 10 200 python -u bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/c5_g$g.log 2>&1 || { echo C5G_FAILED; tail -20 $OUT/c5_g$g.log; exit 1; }
echo "g=$g r=0.65 $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5_g$g.log)"
done
