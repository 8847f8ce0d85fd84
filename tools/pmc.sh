#!/bin/bash
# PMC passes over a reduced bench (one rocprofv3 run per counter group).
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
ARGS=${2:-"--jobs 8 --steps 2 --warmup 1 --no-cpu-baseline"}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/sq -o run -- python -u bench.py $ARGS > $OUT/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python -u bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python -u bench.py $ARGS > $OUT/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq2 -o run -- python -u bench.py $ARGS > $OUT/sq2.log 2>&1
