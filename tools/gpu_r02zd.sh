#!/bin/bash
# Throttle in both producers: GPU tests, then configs 2-5 with the default lib
# and with the throttle compiled out (build/var/libtbc_loff.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02zd
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in 2 3 4 5; do
for v in default loff; do
if [ $v = default ]; then unset TBC_LIB; else export TBC_LIB=$PWD/build/var/libtbc_$v.so; fi
timeout -k 10 240 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c${c}_$v.log 2>&1 || { echo C${c}_${v}_FAILED; tail -20 $OUT/c${c}_$v.log; exit 1; }
echo "c$c $v $(grep -o '"ms_per_step": [0-9.]*' $OUT/c${c}_$v.log) $(grep -o '"data_blocks": [0-9.]*' $OUT/c${c}_$v.log)"
done
done
echo ALL_OK
