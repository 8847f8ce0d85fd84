#!/bin/bash
# Round 2 bench lines: config 1 (replayed benchmark load) and configs 2-5,
# each a separate process under its own time limit, chained with &&.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02d
mkdir -p $OUT
timeout -k 10 500 python -u bench.py --config 1 --steps 3 --warmup 1 > $OUT/c1.log 2>&1 || { echo C1_FAILED; tail -30 $OUT/c1.log; exit 1; }
tail -1 $OUT/c1.log
for c in 2 3 4 5; do
  timeout -k 10 240 python -u bench.py --config $c --steps 10 --warmup 3 > $OUT/c$c.log 2>&1 || { echo C${c}_FAILED; tail -30 $OUT/c$c.log; exit 1; }
  tail -1 $OUT/c$c.log
done
echo BENCH_OK
