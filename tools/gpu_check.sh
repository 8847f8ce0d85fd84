# GPU-box check: parity tests, then bench runs (logs under gpurun_out/).
# usage: gpu_check.sh [CONFIGS...]   (default: 2)
# An ordinary test failure (exit 1) still lets the benches run; a fault,
# abort, segfault or time limit (124/134/137/139 or >128) ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { [ "$1" -ge 124 ]; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" gpurun_out/gpu_tests.log | tail -3; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then echo "TESTS_FAILED rc=$rc"; grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/gpu_tests.log | head -20; fi
if fatal $rc; then exit $rc; fi
for c in ${@:-2}; do
  timeout -k 10 420 python -u bench.py --config $c --steps ${STEPS:-5} --warmup 2 > gpurun_out/bench_c$c.log 2>&1
  brc=$?
  tail -1 gpurun_out/bench_c$c.log | cut -c1-400
  if [ $brc -ne 0 ]; then echo "BENCH_FAILED $c rc=$brc"; tail -20 gpurun_out/bench_c$c.log; fi
  if fatal $brc; then exit $brc; fi
done
exit $rc
