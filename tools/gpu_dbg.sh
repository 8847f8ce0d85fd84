set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dbg
TBC_DEBUG_SYNC=1 timeout -k 10 120 python -u -m pytest tests/test_gpu_grid.py -x -v -s --timeout 100 --timeout-method thread -k chained > gpurun_out/dbg/t1.log 2>&1; echo rc=$? >> gpurun_out/dbg/t1.log
grep -v "^tbc debug: stage .* done" gpurun_out/dbg/t1.log | tail -25
