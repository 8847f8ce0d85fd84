#!/bin/bash
# Sort rewrite: parity tests, then config 3/4/1 bench lines and a config 3 trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02e
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "sort" --timeout 120 --timeout-method thread > $OUT/sort.log 2>&1 || { echo SORT_FAILED; tail -40 $OUT/sort.log; exit 1; }
tail -2 $OUT/sort.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_config1.py -x -v --timeout 300 --timeout-method thread > $OUT/cfg.log 2>&1 || { echo CFG_FAILED; tail -40 $OUT/cfg.log; exit 1; }
tail -2 $OUT/cfg.log
for c in 3 4; do
  timeout -k 10 240 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c$c.log 2>&1 || { echo C${c}_FAILED; tail -30 $OUT/c$c.log; exit 1; }
  tail -1 $OUT/c$c.log | cut -c1-200; grep -o '"kernels_us_per_step.*}' $OUT/c$c.log | cut -c1-300
done
timeout -k 10 300 python -u bench.py --config 1 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c1.log 2>&1 || { echo C1_FAILED; tail -30 $OUT/c1.log; exit 1; }
tail -1 $OUT/c1.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr3 -o run -- python3 -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/tr3.log 2>&1 || { echo TR_FAILED; exit 1; }
echo R02E_OK
