#!/bin/bash
# Round-2 profiles of the current libtbc.so: config 2 (default bench line,
# trace, FETCH/WRITE/SQ PMC passes) with kernel traces of configs 1, 4, 5;
# config 3 and config 5 with their own PMC passes (the sort kernels, the
# throughput regime); the k-way probe trace. Each step under its own limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?usage: profile_r02.sh TAG}
CONFIG=2 EXTRA_CONFIGS="1 4" bash tools/profile.sh ${TAG}_c2 || exit 1
CONFIG=3 bash tools/profile.sh ${TAG}_c3 || exit 1
CONFIG=5 bash tools/profile.sh ${TAG}_c5 || exit 1
mkdir -p gpurun_out/prof_${TAG}_kway
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_kway/trace -o run -- python3 -u tools/scan_probe.py --reps 5 > gpurun_out/prof_${TAG}_kway/probe.log 2>&1 || exit 1
echo PROFILE_R02_OK
