#!/bin/bash
# Round-4 final measurement (through gpurun), in two calls:
#   PART=1: the whole GPU suite, then tools/profile.sh for configs 2, 3, 5
#   PART=2: tools/profile.sh for configs 1 and 4
# (bench line + kernel trace + FETCH_SIZE / WRITE_SIZE / SQ passes each, every
# GPU step under its own time limit, chained by &&). Summarise afterwards on
# the CPU with tools/collect_r04.sh.
set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_r04.log 2>&1
  tail -1 gpurun_out/gpu_tests_r04.log
  for c in 2 3 5; do CONFIG=$c bash tools/profile.sh r04_c$c; done
else
  for c in 1 4; do CONFIG=$c bash tools/profile.sh r04_c$c; done
fi
md5sum tigerbeetle_amd/libtbc.so
echo R04_OK
