#!/bin/bash
# Config 1 bench line only (optional trace): tools/gpu_c1.sh [trace]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/c1
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --config 1 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c1.log 2>&1 || { echo C1_FAILED; tail -30 $OUT/c1.log; exit 1; }
tail -1 $OUT/c1.log | cut -c1-200; grep -o '"kernels_us_per_step[^}]*}' $OUT/c1.log
if [ "$1" = trace ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o run -- python3 -u bench.py --config 1 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/tr.log 2>&1 || { echo TR_FAILED; exit 1; }
fi
echo C1_OK
