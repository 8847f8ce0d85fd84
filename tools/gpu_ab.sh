# GPU-box A/B runs: each argument is "TAG|ENV|ARGS" -> bench.py ARGS under ENV,
# the line into gpurun_out/ab_TAG.log. Stops at the first fault or time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  IFS='|' read -r tag envs args <<< "$spec"
  env $envs timeout -k 10 300 python -u bench.py $args > gpurun_out/ab_$tag.log 2>&1
  rc=$?
  echo "$tag rc=$rc $(tail -1 gpurun_out/ab_$tag.log | python3 -c 'import json,sys
try:
  d=json.loads(sys.stdin.read()); print(d["ms_per_step"], json.dumps(d.get("kernels_us_per_step")))
except Exception as e: print("?")')"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
