#!/bin/bash
# Sort variants by kernel trace: the memtable sort's kernels of configs 3 and 4
# (default lib: round-robin tiles, resident grid, 8-deep look-back; k16: 16-deep
# look-back + neighbour-lane pack; sortold: before round 2d).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02zi
mkdir -p $OUT
for c in 3 4; do
for v in default k16 sortold; do
if [ $v = default ]; then unset TBC_LIB; else export TBC_LIB=$PWD/build/var/libtbc_$v.so; fi
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t_c${c}_$v -o run -- python3 -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $OUT/t_c${c}_$v.log 2>&1 || { echo T_${c}_${v}_FAILED; tail -20 $OUT/t_c${c}_$v.log; exit 1; }
echo "c$c $v $(grep -o '"ms_per_step": [0-9.]*' $OUT/t_c${c}_$v.log)"
done
done
echo ALL_OK
