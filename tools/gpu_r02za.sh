#!/bin/bash
# Producer throttle / streamed window loads: config 2 step time and k_data_blocks
# FETCH_SIZE per library variant (build/var/libtbc_*.so, built with -D flags).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02za
mkdir -p $OUT
for v in loff l12 l8 l64 nt12 nt6; do
export TBC_LIB=$PWD/build/var/libtbc_$v.so
timeout -k 10 200 python -u bench.py --config 2 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c2_$v.log 2>&1 || { echo C2_${v}_FAILED; tail -20 $OUT/c2_$v.log; exit 1; }
echo "$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/c2_$v.log) $(grep -o '"data_blocks": [0-9.]*' $OUT/c2_$v.log)"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$v -o run -- python3 -u bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/fetch_$v.log 2>&1 || { echo FETCH_${v}_FAILED; tail -20 $OUT/fetch_$v.log; exit 1; }
done
echo ALL_OK
