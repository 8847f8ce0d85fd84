#!/bin/bash
# Round-2d: full GPU suite + smoke, then config 2 profile (+ traces of configs 1 and 4).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02d
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02d/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02d/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02d/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02d/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r02d/smoke.log; exit 1; }
tail -1 gpurun_out/r02d/smoke.log
CONFIG=2 EXTRA_CONFIGS="1 4" bash tools/profile.sh r02d_c2 || exit 1
echo PART1_OK
