#!/bin/bash
# Column-pair chains: parity tests (throughput regime), config 5 with and without col2.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02x
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_col2.py -x -v --timeout 200 --timeout-method thread > $OUT/col2.log 2>&1 || { echo COL2_FAILED; tail -40 $OUT/col2.log; exit 1; }
tail -4 $OUT/col2.log
timeout -k 10 200 python -u bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/c5.log 2>&1 || { echo C5_FAILED; tail -20 $OUT/c5.log; exit 1; }
echo "c5 $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/c5.log)"
TBC_NO_COL2=1 timeout -k 10 200 python -u bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/c5n.log 2>&1 || { echo C5N_FAILED; tail -20 $OUT/c5n.log; exit 1; }
echo "c5n $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5n.log) $(grep -o '"kernels_us_per_step[^}]*}' $OUT/c5n.log)"
