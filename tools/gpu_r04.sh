# Round 4 GPU call: parity tests (changed areas first), then config 2 bench
# variants (pipelined depth 3; fused, depth 1; tail chain packing A/B).
# Logs under gpurun_out/r04/. Fatal exits (>=124) end the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04${TAG:-}
mkdir -p $O
fatal() { [ "$1" -ge 124 ]; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_overlap.py tests/test_gpu_unique.py tests/test_gpu_engine.py tests/test_manifest.py ${EXTRA_TESTS:-} -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests_new.log 2>&1
  rc=$?; tail -2 $O/tests_new.log
  if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" $O/tests_new.log | head -20; exit $rc; fi
  if [ -z "$SKIP_ALL" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests_all.log 2>&1
  rc=$?; tail -2 $O/tests_all.log
  if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" $O/tests_all.log | head -20; exit $rc; fi
  fi
fi
run() { # name env... -- args
  local name=$1; shift
  timeout -k 10 300 env "$@" > $O/bench_$name.log 2>&1
  local brc=$?
  echo "== $name rc=$brc"; grep '^{' $O/bench_$name.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); k=d.get('kernels_us_per_step',{}); p=d.get('pcie',{})
    print(' ms/step', d['ms_per_step'], 'MB/s', d['value'], 'frac', d['roofline']['frac'], 'dom', d['roofline'].get('kernel') or d['roofline']['dominant_kernel']['kernel'], {a:b for a,b in k.items()}, 'd2h', p.get('d2h',{}).get('GBps'), 'h2d', p.get('h2d',{}).get('GBps'), 'incl', p.get('pcie_inclusive_MBps'), 'staged', p.get('staged'))
"
  if [ $brc -ne 0 ]; then tail -15 $O/bench_$name.log; fi
  return $brc
}
B="python -u bench.py --steps ${STEPS:-20} --warmup 5"
for v in ${VARIANTS:-d3 d1 d2 t8 t16}; do
  case $v in
    d3) run d3 $B --depth 3 ;;
    d1) run d1 $B --depth 1 --no-cpu-baseline ;;
    d2) run d2 $B --depth 2 --no-cpu-baseline ;;
    d4) run d4 $B --depth 4 --no-cpu-baseline ;;
    t8) run t8 TBC_TAIL_CHAINS=8 $B --depth 3 --no-cpu-baseline ;;
    t16) run t16 TBC_TAIL_CHAINS=16 $B --depth 3 --no-cpu-baseline ;;
    t4) run t4 TBC_TAIL_CHAINS=4 $B --depth 3 --no-cpu-baseline ;;
    tv) run tv TBC_TAIL_STEP=valu $B --depth 3 --no-cpu-baseline ;;
    p1) run p1 $B --depth 1 --pipeline on --no-cpu-baseline ;;
    p3) run p3 $B --depth 3 --pipeline on --no-cpu-baseline ;;
    h3) run h3 TBC_TAIL_TABLES=64 $B --depth 3 --no-cpu-baseline ;;
    h8) run h8 TBC_TAIL_TABLES=64 TBC_TAIL_CHAINS=8 $B --depth 3 --no-cpu-baseline ;;
    h16) run h16 TBC_TAIL_TABLES=64 TBC_TAIL_CHAINS=16 $B --depth 3 --no-cpu-baseline ;;
    h4) run h4 TBC_TAIL_TABLES=64 TBC_TAIL_CHAINS=4 $B --depth 3 --no-cpu-baseline ;;
    c5h) run c5h TBC_TAIL_TABLES=64 $B --depth 3 --config 5 --no-cpu-baseline ;;
    c1) run c1 $B --config 1 --steps 3 --warmup 1 --no-cpu-baseline ;;
    c1h) run c1h TBC_TAIL_TABLES=64 $B --config 1 --steps 3 --warmup 1 --no-cpu-baseline ;;
    fp3) run fp3 TBC_FRONT_PRIORITY=1 $B --depth 3 --no-cpu-baseline ;;
    fp5) run fp5 TBC_FRONT_PRIORITY=1 $B --depth 3 --config 5 --no-cpu-baseline ;;
    d4p) run d4p $B --depth 4 --no-cpu-baseline ;;
    c51) run c51 $B --depth 1 --config 5 --no-cpu-baseline ;;
    c1ns) run c1ns TBC_NO_SPECULATION=1 $B --config 1 --steps 3 --warmup 1 --no-cpu-baseline ;;
    c1u) run c1u TBC_UPLOAD_COPY=1 $B --config 1 --steps 3 --warmup 1 --no-cpu-baseline ;;
    c1gs) run c1gs TBC_GRID_SPECULATION=1 $B --config 1 --steps 3 --warmup 1 --no-cpu-baseline ;;
    c3) run c3 $B --depth 3 --config 3 --no-cpu-baseline ;;
    c4) run c4 $B --depth 3 --config 4 --no-cpu-baseline ;;
    c5) run c5 $B --depth 3 --config 5 --no-cpu-baseline ;;
  esac
  r=$?; if fatal $r; then exit $r; fi
done
echo DONE_OK
