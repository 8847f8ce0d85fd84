# GPU-box check: parity tests, then bench runs (logs under gpurun_out/).
# usage: gpu_check.sh [CONFIGS...]   (default: 2)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
for c in ${@:-2}; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 > gpurun_out/bench_c$c.log 2>&1 || { echo BENCH_FAILED $c; tail -30 gpurun_out/bench_c$c.log; exit 1; }
  tail -1 gpurun_out/bench_c$c.log
done
