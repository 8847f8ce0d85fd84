#!/bin/bash
# Copy loops with loads in flight: parity (configs, sort, parity), then config 5 (groups 1/3) and configs 2/3/4 lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02h
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { echo T_FAILED; tail -40 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for g in 1 3; do
  TBC_GROUPS=$g timeout -k 10 240 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c5g$g.log 2>&1 || { echo G${g}_FAILED; tail -20 $OUT/c5g$g.log; exit 1; }
  echo "c5 groups=$g $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5g$g.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/c5g$g.log)"
done
for c in 2 3 4; do
  timeout -k 10 240 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c$c.log 2>&1 || { echo C${c}_FAILED; tail -20 $OUT/c$c.log; exit 1; }
  echo "c$c $(grep -o '"ms_per_step": [0-9.]*' $OUT/c$c.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/c$c.log)"
done
