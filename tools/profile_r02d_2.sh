#!/bin/bash
# Round-2d profiles, part 2: configs 3 and 5 (bench line, trace, PMC passes), k-way probe trace.
set -o pipefail
mkdir -p gpurun_out/r02d
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CONFIG=3 bash tools/profile.sh r02d_c3 || exit 1
CONFIG=5 bash tools/profile.sh r02d_c5 || exit 1
mkdir -p gpurun_out/prof_r02d_kway
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02d_kway/trace -o run -- python3 -u tools/scan_probe.py --reps 5 > gpurun_out/prof_r02d_kway/probe.log 2>&1 || exit 1
echo PART2_OK
for c in 1 4; do
timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 > gpurun_out/r02d/bench_c$c.log 2>&1 || { echo C${c}_FAILED; tail -20 gpurun_out/r02d/bench_c$c.log; exit 1; }
done
echo BENCH_OK
