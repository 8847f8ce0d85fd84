#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats) of bench configs, one
# process each under its own time limit: tools/gpu_trace.sh TAG CONFIG...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?usage: gpu_trace.sh TAG CONFIG...}
shift
OUT=gpurun_out/trace_$TAG
mkdir -p $OUT
for c in "$@"; do
  steps="--steps 5 --warmup 2"
  [ "$c" = 1 ] && steps="--steps 1 --warmup 1"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c$c -o run -- python3 -u bench.py --config $c $steps --no-cpu-baseline > $OUT/c$c.log 2>&1 || { echo TRACE_C${c}_FAILED; tail -20 $OUT/c$c.log; exit 1; }
  tail -1 $OUT/c$c.log | cut -c1-300
done
echo TRACE_OK
