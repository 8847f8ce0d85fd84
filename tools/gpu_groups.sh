#!/bin/bash
# A/B of job-group counts for throughput-regime batches (config 5).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/groups
mkdir -p $OUT
for g in 1 2 3 4; do
  TBC_GROUPS=$g timeout -k 10 240 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/g$g.log 2>&1 || { echo G${g}_FAILED; tail -20 $OUT/g$g.log; exit 1; }
  echo "groups=$g $(grep -o '"ms_per_step": [0-9.]*' $OUT/g$g.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/g$g.log)"
done
