#!/bin/bash
# Round-3 final measurement of the current libtbc.so (through gpurun): the
# GPU test suite, then configs 2, 5 and 3 through tools/profile.sh (bench
# line with CPU baseline, kernel trace, FETCH/WRITE/SQ PMC passes, each a run
# of its own), bench lines and kernel traces of configs 1 and 4, and the
# scan-path k-way probe. Every GPU step has its own time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r03/gpu_tests.log 2>&1 || { tail -5 gpurun_out/r03/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03/gpu_tests.log
for c in 2 5 3; do
  CONFIG=$c bash tools/profile.sh r03_c$c > gpurun_out/r03/profile_c$c.log 2>&1 || { echo PROFILE_FAILED $c; tail -5 gpurun_out/r03/profile_c$c.log; exit 1; }
  tail -1 gpurun_out/prof_r03_c$c/bench.json | cut -c1-160
done
for c in 1 4; do
  S=20; W=3; [ $c = 1 ] && { S=5; W=1; }
  timeout -k 10 400 python -u bench.py --config $c --steps $S --warmup $W > gpurun_out/r03/bench_c$c.log 2>&1 || { echo BENCH_FAILED $c; exit 1; }
  tail -1 gpurun_out/r03/bench_c$c.log | cut -c1-160
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03/trace_c$c -o run -- python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03/trace_c$c.log 2>&1 || { echo TRACE_FAILED $c; exit 1; }
done
timeout -k 10 120 python -u tools/scan_probe.py > gpurun_out/r03/scan_probe.json 2> gpurun_out/r03/scan_probe.log || exit 1
md5sum tigerbeetle_amd/libtbc.so > gpurun_out/r03/lib.md5
echo R03_OK
