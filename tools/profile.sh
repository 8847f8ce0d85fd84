#!/bin/bash
# One round's measurement on the GPU box (run through gpurun):
#   1. bench.py default line (with the CPU baseline)        -> bench.json
#   2. rocprofv3 --kernel-trace --stats over the same bench  -> trace/
#   3. one --pmc pass per TCC counter (FETCH_SIZE, WRITE_SIZE), each its own
#      run (MI355X_MICROARCH.md: they do not fit one pass)   -> fetch/, write/
# Every GPU step has its own time limit and the steps are chained with &&.
# Summarise afterwards on the CPU with tools/traffic.py.
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:?usage: profile.sh TAG}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
CFG=${CONFIG:-2}
ARGS="--config $CFG --steps 10 --warmup 3 ${BENCH_ARGS:-}"
SHORT="--config $CFG --steps 3 --warmup 1 ${BENCH_ARGS:-}"
timeout -k 10 240 python -u bench.py $ARGS > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log > $OUT/bench.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 -u bench.py $ARGS --no-cpu-baseline > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 -u bench.py $SHORT --no-cpu-baseline > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 -u bench.py $SHORT --no-cpu-baseline > $OUT/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/sq -o run -- python3 -u bench.py $SHORT --no-cpu-baseline > $OUT/sq.log 2>&1
md5sum tigerbeetle_amd/libtbc.so > $OUT/lib.md5
echo PROFILE_OK
# Kernel traces of the other BASELINE configs (no PMC passes).
for c in $EXTRA_CONFIGS; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c$c -o run -- python3 -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $OUT/trace_c$c.log 2>&1
done
echo PROFILE_EXTRA_OK
