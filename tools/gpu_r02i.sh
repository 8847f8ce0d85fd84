#!/bin/bash
# Assembling merge (throughput regime, pipelined and values-only batches): parity, then config 5/1 lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02i
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_grid.py tests/test_gpu_split.py -x -v --timeout 200 --timeout-method thread > $OUT/t1.log 2>&1 || { echo T1_FAILED; grep -n "PASS\|FAIL\|Error\|tbc" $OUT/t1.log | tail -30; exit 1; }
tail -1 $OUT/t1.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_config1.py -x -q --timeout 250 --timeout-method thread > $OUT/t2.log 2>&1 || { echo T2_FAILED; tail -30 $OUT/t2.log; exit 1; }
tail -1 $OUT/t2.log
for v in "TBC_GROUPS=1" ""; do
  env $v timeout -k 10 240 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c5.log 2>&1 || { echo C5_FAILED; tail -20 $OUT/c5.log; exit 1; }
  echo "c5 $v $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/c5.log)"
done
timeout -k 10 300 python -u bench.py --config 1 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c1.log 2>&1 || { echo C1_FAILED; tail -20 $OUT/c1.log; exit 1; }
echo "c1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/c1.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/c1.log)"
