#!/bin/bash
# Config 2 bench: speculated (default) vs TBC_NO_SPECULATION=1; config 3 and 4 lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02n
mkdir -p $OUT
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c2.log 2>&1 || { echo C2_FAILED; tail -20 $OUT/c2.log; exit 1; }
TBC_NO_SPECULATION=1 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c2_nospec.log 2>&1 || { echo C2N_FAILED; tail -20 $OUT/c2_nospec.log; exit 1; }
timeout -k 10 200 python -u bench.py --config 3 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c3.log 2>&1 || { echo C3_FAILED; tail -20 $OUT/c3.log; exit 1; }
timeout -k 10 200 python -u bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4.log 2>&1 || { echo C4_FAILED; tail -20 $OUT/c4.log; exit 1; }
for f in c2 c2_nospec c3 c4; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $OUT/$f.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/$f.log)"; done
