#!/bin/bash
# UNIQUE_KEYS speculation: its tests, then the parity suite that touches the block phase.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02m
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_unique.py -x -v --timeout 120 --timeout-method thread > $OUT/unique.log 2>&1 || { echo UNIQUE_FAILED; tail -40 $OUT/unique.log; exit 1; }
tail -3 $OUT/unique.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { echo PARITY_FAILED; tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
