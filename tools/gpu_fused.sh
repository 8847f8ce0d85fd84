#!/bin/bash
# A/B: config 5 with the fused (producers + chains) block kernel in the throughput regime.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/fused
mkdir -p $OUT
for v in "TBC_GROUPS=1" "TBC_GROUPS=1 TBC_FUSED_MAX_WAVES=100000" "TBC_GROUPS=3 TBC_FUSED_MAX_WAVES=100000"; do
  env $v timeout -k 10 240 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/run.log 2>&1 || { echo FAILED $v; tail -20 $OUT/run.log; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/run.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/run.log)"
done
