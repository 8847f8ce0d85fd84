#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/kwaydbg
mkdir -p $OUT
timeout -k 10 120 python -u -m pytest tests/test_gpu_kway.py -x -v -s --timeout 100 --timeout-method thread > $OUT/t.log 2>&1
echo rc=$?
grep -n "tbc\|PASS\|FAIL\|Error" $OUT/t.log | head -40
