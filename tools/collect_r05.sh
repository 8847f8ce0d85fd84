#!/bin/bash
# Copy what tools/profile_r05.sh left under gpurun_out/ into profiles/ (run
# here, after the gpurun calls): per config traffic.json (md5 of the measured
# libtbc.so), kernel stats and the bench line (tools/traffic.py), and the GPU
# suite's summary.
set -e -o pipefail
cd "$(dirname "$0")/.."
for c in ${CONFIGS:-1 2 3 4 5}; do
  [ -d gpurun_out/prof_r05_c$c ] || continue
  rm -rf profiles/r05_c$c
  python tools/traffic.py gpurun_out/prof_r05_c$c profiles/r05_c$c
done
true
