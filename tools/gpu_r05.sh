#!/bin/bash
# Round-5 GPU call: optional test selection, then bench variants.
#   TESTS="<pytest args>" (empty: skip tests)   RUNS="name|ENV=.. ENV2=..|bench args;..."
# Each GPU step has its own time limit; a fault, abort, segfault or time
# limit (exit >= 124) ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest $TESTS -x -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?
  grep -cE "PASSED" $OUT/tests.log; tail -2 $OUT/tests.log
  if [ $rc -ne 0 ]; then echo "TESTS_FAILED rc=$rc"; grep -E "^(FAILED|ERROR)|Error|assert" $OUT/tests.log | head -20; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
fi
IFS=';' read -ra SPECS <<< "$RUNS"
for spec in "${SPECS[@]}"; do
  [ -z "$spec" ] && continue
  IFS='|' read -r name envs args <<< "$spec"
  env $envs timeout -k 10 ${BENCH_LIMIT:-300} python -u bench.py $args > $OUT/bench_$name.log 2>&1
  brc=$?
  echo "== $name: $(tail -1 $OUT/bench_$name.log | python3 -c 'import sys,json
try:
  d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms", d.get("kernels_us_per_step"))
except Exception as e: print("no json")')"
  if [ $brc -ne 0 ]; then echo "BENCH_FAILED $name rc=$brc"; tail -15 $OUT/bench_$name.log; fi
  if [ $brc -ge 124 ]; then exit $brc; fi
done
echo CALL_DONE
