#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/kway
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kway.py -x -v --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { echo KWAY_FAILED; tail -40 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
timeout -k 10 200 python -u tools/scan_probe.py > $OUT/probe.log 2>&1 || { echo PROBE_FAILED; tail -20 $OUT/probe.log; exit 1; }
tail -1 $OUT/probe.log
timeout -k 10 200 python -u tools/scan_probe.py --streams 16 --per-stream 1000000 > $OUT/probe16.log 2>&1 && tail -1 $OUT/probe16.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o run -- python3 -u tools/scan_probe.py --reps 5 > $OUT/tr.log 2>&1 || { echo TR_FAILED; exit 1; }
echo KWAY_OK
