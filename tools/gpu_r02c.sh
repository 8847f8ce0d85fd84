set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02c
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "sort" --timeout 120 --timeout-method thread > gpurun_out/r02c/sort.log 2>&1 || { echo SORT_FAILED; tail -60 gpurun_out/r02c/sort.log; exit 1; }
tail -3 gpurun_out/r02c/sort.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_config1.py -x -v -s --timeout 560 --timeout-method thread > gpurun_out/r02c/config1.log 2>&1 || { echo C1_FAILED; tail -60 gpurun_out/r02c/config1.log; exit 1; }
tail -5 gpurun_out/r02c/config1.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r02c/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02c/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r02c/gpu_tests.log
