#!/bin/bash
# Sort passes with tiles interleaved across tables: sort tests, configs 3 and 4
# A/B against the previous order (build/var/libtbc_sortold.so), and a kernel
# trace of config 3 for the pass times.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02zh
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1; do
for c in 3 4; do
for v in default inter sortold; do
if [ $v = default ]; then unset TBC_LIB; else export TBC_LIB=$PWD/build/var/libtbc_$v.so; fi
timeout -k 10 240 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c${c}_${v}_$rep.log 2>&1 || { echo C${c}_${v}_FAILED; tail -20 $OUT/c${c}_${v}_$rep.log; exit 1; }
echo "c$c $v $rep $(grep -o '"ms_per_step": [0-9.]*' $OUT/c${c}_${v}_$rep.log)"
done
done
done
unset TBC_LIB
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c3 -o run -- python3 -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/trace_c3.log 2>&1 || { echo TRACE_FAILED; tail -20 $OUT/trace_c3.log; exit 1; }
echo ALL_OK
