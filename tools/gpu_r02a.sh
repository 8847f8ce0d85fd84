set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02a
timeout -k 10 240 ./tools/aegis_lab 16384 > gpurun_out/r02a/aegis_lab.json 2>&1 || { echo LAB_FAILED; tail -20 gpurun_out/r02a/aegis_lab.json; exit 1; }
tail -3 gpurun_out/r02a/aegis_lab.json
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02a/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02a/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r02a/gpu_tests.log
