#!/bin/bash
# Pipelined grid batches: grid + config 1 parity, full GPU suite, config 1/2 bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02f
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -x -v --timeout 120 --timeout-method thread > $OUT/grid.log 2>&1 || { echo GRID_FAILED; tail -40 $OUT/grid.log; exit 1; }
tail -2 $OUT/grid.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_config1.py -x -v -s --timeout 300 --timeout-method thread > $OUT/c1t.log 2>&1 || { echo C1T_FAILED; tail -40 $OUT/c1t.log; exit 1; }
tail -2 $OUT/c1t.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/all.log 2>&1 || { echo ALL_FAILED; tail -40 $OUT/all.log; exit 1; }
tail -2 $OUT/all.log
timeout -k 10 300 python -u bench.py --config 1 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c1.log 2>&1 || { echo C1_FAILED; tail -30 $OUT/c1.log; exit 1; }
tail -1 $OUT/c1.log | cut -c1-200; grep -o '"kernels_us_per_step[^}]*}' $OUT/c1.log
echo R02F_OK
