set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02b
TBC_DEBUG_SYNC=1 timeout -k 5 60 python -u tools/dbg/grid_dbg.py disk > gpurun_out/r02b/dbg_disk.log 2>&1 || { echo DBG_FAILED; cat gpurun_out/r02b/dbg_disk.log; exit 1; }
cat gpurun_out/r02b/dbg_disk.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02b/grid.log 2>&1 || { echo GRID_FAILED; tail -60 gpurun_out/r02b/grid.log; exit 1; }
tail -5 gpurun_out/r02b/grid.log
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r02b/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02b/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r02b/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02b/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/r02b/bench.log; exit 1; }
tail -1 gpurun_out/r02b/bench.log
