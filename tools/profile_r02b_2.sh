#!/bin/bash
# Round-2b profiles, part 2: configs 3 and 5 (bench line, trace, PMC passes), k-way probe trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CONFIG=3 bash tools/profile.sh r02b_c3 || exit 1
CONFIG=5 bash tools/profile.sh r02b_c5 || exit 1
mkdir -p gpurun_out/prof_r02b_kway
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02b_kway/trace -o run -- python3 -u tools/scan_probe.py --reps 5 > gpurun_out/prof_r02b_kway/probe.log 2>&1 || exit 1
echo PART2_OK
