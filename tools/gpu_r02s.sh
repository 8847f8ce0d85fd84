#!/bin/bash
# Chains alone in the fused kernel (bodies assembled first, merge path) vs the normal fused kernel, config 2.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02s
mkdir -p $OUT
TBC_NO_SPECULATION=1 TBC_PROBE_CHAINS_ALONE=1 timeout -k 10 200 python -u bench.py --config 2 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/ca2.log 2>&1 || { echo CA_FAILED; tail -20 $OUT/ca2.log; exit 1; }
echo "ca2 $(grep -o '"kernels_us_per_step[^}]*}' $OUT/ca2.log)"
TBC_NO_SPECULATION=1 timeout -k 10 200 python -u bench.py --config 2 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/ns2.log 2>&1 || { echo NS_FAILED; tail -20 $OUT/ns2.log; exit 1; }
echo "ns2 $(grep -o '"kernels_us_per_step[^}]*}' $OUT/ns2.log)"
