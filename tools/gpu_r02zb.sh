#!/bin/bash
# L2 hit/miss and raw read requests of k_data_blocks on config 2, with and
# without the producer throttle (calibrates FETCH_SIZE for the chains' dword reads).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02zb
mkdir -p $OUT
for v in loff l12; do
export TBC_LIB=$PWD/build/var/libtbc_$v.so
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/hit_$v -o run -- python3 -u bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/hit_$v.log 2>&1 || { echo HIT_${v}_FAILED; tail -20 $OUT/hit_$v.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $OUT/rd_$v -o run -- python3 -u bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/rd_$v.log 2>&1 || { echo RD_${v}_FAILED; tail -20 $OUT/rd_$v.log; exit 1; }
done
echo ALL_OK
