# GPU-box: the AEGIS layout lab (tools/aegis_lab.hip, built here beforehand).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 ./tools/aegis_lab ${1:-4096} > gpurun_out/aegis_lab.json 2>&1 || { echo LAB_FAILED; tail -20 gpurun_out/aegis_lab.json; exit 1; }
grep -E '"messages": (2|1008|2016|4096),' gpurun_out/aegis_lab.json | grep -E 'prod-valukey|halves64'
tail -1 gpurun_out/aegis_lab.json
