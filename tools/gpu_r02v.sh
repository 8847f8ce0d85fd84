#!/bin/bash
# Chains with the acquire-once progress check: unique + parity tests, config 2 (spec, nospec, chains alone).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02v
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_unique.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 200 python -u bench.py --config 2 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c2.log 2>&1 || { echo C2_FAILED; tail -20 $OUT/c2.log; exit 1; }
echo "c2 $(grep -o '"ms_per_step": [0-9.]*' $OUT/c2.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/c2.log)"
TBC_NO_SPECULATION=1 TBC_PROBE_CHAINS_ALONE=1 timeout -k 10 200 python -u bench.py --config 2 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/ca2.log 2>&1 || { echo CA_FAILED; tail -20 $OUT/ca2.log; exit 1; }
echo "ca2 $(grep -o '"kernels_us_per_step[^}]*}' $OUT/ca2.log)"
TBC_NO_SPECULATION=1 timeout -k 10 200 python -u bench.py --config 2 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/ns2.log 2>&1 || { echo NS_FAILED; tail -20 $OUT/ns2.log; exit 1; }
echo "ns2 $(grep -o '"ms_per_step": [0-9.]*' $OUT/ns2.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/ns2.log)"
