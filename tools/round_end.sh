#!/bin/bash
# Round-end check of the current libtbc.so (through gpurun): the whole GPU
# test suite, then the profile (tools/profile_final.sh) and a 16-stream
# k-way probe. Each GPU step has its own time limit; steps chained by &&.
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:?usage: round_end.sh TAG}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
tail -1 gpurun_out/gpu_tests_$TAG.log
EXTRA_CONFIGS="3 4 5" bash tools/profile_final.sh $TAG
timeout -k 10 120 python -u tools/scan_probe.py --streams 16 --per-stream 1000000 --tree transfers.debit_account_id > gpurun_out/prof_$TAG/scan_probe_16.json
echo ROUND_END_OK
