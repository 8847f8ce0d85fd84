#!/bin/bash
# Round-5 final measurement (through gpurun), in two calls:
#   PART=1: tools/profile.sh for configs 2, 3, 5 (the GPU suite runs in a call of its own)
#   PART=2: tools/profile.sh for configs 1 and 4
# (bench line + kernel trace + FETCH_SIZE / WRITE_SIZE / SQ passes each, every
# GPU step under its own time limit, chained by &&). Summarise afterwards on
# the CPU with tools/collect_r05.sh.
set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${PART:-1}" = 1 ]; then
  for c in 2 3 5; do CONFIG=$c bash tools/profile.sh r05_c$c; done
else
  for c in 1 4; do CONFIG=$c bash tools/profile.sh r05_c$c; done
  # Config 4's key-range split rehearsed with two ranks on this one GPU
  # (timing over gloo), beside its N = 1 line.
  TBC_BENCH_SAME_DEVICE=1 TBC_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29537 bench.py --gpus 2 --config 4 --steps 10 \
    --warmup 3 --no-cpu-baseline > gpurun_out/split_c4_n2.log 2>&1
  grep '^{' gpurun_out/split_c4_n2.log | tail -1
fi
md5sum tigerbeetle_amd/libtbc.so
echo R05_OK
