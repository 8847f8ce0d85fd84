#!/bin/bash
# Truncated sort: sort parity tests, config 3/4 and config 1 bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02j
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "sort" --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { echo T_FAILED; grep -n "PASS\|FAIL\|Error\|tbc" $OUT/t.log | tail -30; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_config1.py -x -q --timeout 300 --timeout-method thread > $OUT/t2.log 2>&1 || { echo T2_FAILED; tail -30 $OUT/t2.log; exit 1; }
tail -1 $OUT/t2.log
for c in 3 4; do
  timeout -k 10 240 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c$c.log 2>&1 || { echo C${c}_FAILED; tail -20 $OUT/c$c.log; exit 1; }
  echo "c$c $(grep -o '"ms_per_step": [0-9.]*' $OUT/c$c.log)"
done
timeout -k 10 300 python -u bench.py --config 1 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c1.log 2>&1 || { echo C1_FAILED; tail -20 $OUT/c1.log; exit 1; }
echo "c1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/c1.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/c1.log)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr1 -o run -- python3 -u bench.py --config 1 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/tr1.log 2>&1 || { echo TR_FAILED; exit 1; }
echo R02J_OK
