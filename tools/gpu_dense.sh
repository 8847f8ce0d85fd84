#!/bin/bash
# A/B: dense vs spread chain packing in pipelined throughput-regime tails (config 5).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/dense
mkdir -p $OUT
for v in "TBC_SPREAD_CHAINS=1" "TBC_GROUPS=4" "TBC_GROUPS=2" "TBC_GROUPS=6" "TBC_GROUPS=8"; do
  env $v timeout -k 10 240 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/run.log 2>&1 || { echo FAILED $v; tail -20 $OUT/run.log; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/run.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/run.log)"
done
