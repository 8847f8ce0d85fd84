#!/bin/bash
# Grouped (pipelined) throughput-regime batches: config tests, config 5/2 bench lines, config 5 trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02g
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $OUT/cfg.log 2>&1 || { echo CFG_FAILED; tail -40 $OUT/cfg.log; exit 1; }
tail -2 $OUT/cfg.log
for c in 5 2; do
  timeout -k 10 240 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c$c.log 2>&1 || { echo C${c}_FAILED; tail -30 $OUT/c$c.log; exit 1; }
  tail -1 $OUT/c$c.log | cut -c1-200; grep -o '"kernels_us_per_step[^}]*}' $OUT/c$c.log
done
TBC_NO_GROUPS=1 timeout -k 10 240 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c5_nogroups.log 2>&1 || { echo C5NG_FAILED; exit 1; }
tail -1 $OUT/c5_nogroups.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr5 -o run -- python3 -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/tr5.log 2>&1 || { echo TR_FAILED; exit 1; }
echo R02G_OK
