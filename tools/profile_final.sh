#!/bin/bash
# Round-end measurement of the current libtbc.so (through gpurun): config 2
# bench + kernel trace + FETCH/WRITE PMC passes (tools/profile.sh), then the
# scan-path k-way merge probe alone and under a kernel trace.
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:?usage: profile_final.sh TAG}
bash tools/profile.sh $TAG
OUT=gpurun_out/prof_$TAG
timeout -k 10 180 python -u tools/scan_probe.py > $OUT/scan_probe.json 2> $OUT/scan_probe.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_kway -o run -- python3 -u tools/scan_probe.py --reps 5 > $OUT/trace_kway.log 2>&1
echo FINAL_OK
