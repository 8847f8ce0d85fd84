#!/bin/bash
# Speculated-producer throttle A/B, interleaved twice: configs 2 and 4 with the
# default lib and with the throttle compiled out (build/var/libtbc_loff.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02ze
mkdir -p $OUT
for rep in 1 2; do
for c in 2 4; do
for v in default loff; do
if [ $v = default ]; then unset TBC_LIB; else export TBC_LIB=$PWD/build/var/libtbc_$v.so; fi
timeout -k 10 240 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c${c}_${v}_$rep.log 2>&1 || { echo C${c}_${v}_FAILED; tail -20 $OUT/c${c}_${v}_$rep.log; exit 1; }
echo "c$c $v $rep $(grep -o '"ms_per_step": [0-9.]*' $OUT/c${c}_${v}_$rep.log) $(grep -o '"data_blocks": [0-9.]*' $OUT/c${c}_${v}_$rep.log)"
done
done
done
echo ALL_OK
