# Round-6 GPU call: targeted tests first (fail fast), then the whole GPU
# suite, then driver-shaped config-2 bench lines. Logs under gpurun_out/$TAG.
# usage: gpu_r06.sh TAG [pytest -k selection for the first step]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?tag}
SEL=${2:-}
mkdir -p gpurun_out/$TAG
fatal() { [ "$1" -ge 124 ]; }
if [ -n "$SEL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$SEL" > gpurun_out/$TAG/first.log 2>&1
  rc=$?; tail -3 gpurun_out/$TAG/first.log
  if [ $rc -ne 0 ]; then echo "FIRST_FAILED rc=$rc"; grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/$TAG/first.log | head -20; exit $rc; fi
fi
if [ -z "$NO_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/$TAG/tests.log 2>&1
  rc=$?; tail -2 gpurun_out/$TAG/tests.log
  if [ $rc -ne 0 ]; then echo "TESTS_FAILED rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/$TAG/tests.log | head -20; fi
  if fatal $rc; then exit $rc; fi
fi
for c in ${CONFIGS:-2}; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 > gpurun_out/$TAG/bench_c${c}_20.log 2>&1
  brc=$?; tail -1 gpurun_out/$TAG/bench_c${c}_20.log | cut -c1-300; echo
  if fatal $brc; then exit $brc; fi
done
if [ -n "$BENCH_DEFAULT" ]; then
  timeout -k 10 300 python -u bench.py > gpurun_out/$TAG/bench_default.log 2>&1
  tail -1 gpurun_out/$TAG/bench_default.log | cut -c1-300; echo
fi
exit ${rc:-0}
