#!/bin/bash
# L2 read requests of k_data_blocks on config 2 with producers only / chains only
# (TBC_PROBE_*), to split the full kernel's misses between producers and chains.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02zc
mkdir -p $OUT
for v in PRODUCERS_ONLY CHAINS_ALONE; do
export TBC_PROBE_$v=1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d $OUT/$v -o run -- python3 -u bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/$v.log 2>&1 || { echo ${v}_FAILED; tail -20 $OUT/$v.log; exit 1; }
unset TBC_PROBE_$v
done
echo ALL_OK
