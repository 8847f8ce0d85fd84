# A/B bench lines on one box: each variant is "label|env assignments|bench args"
# (one per line on stdin); each runs under its own time limit, logs under
# gpurun_out/$TAG/ab_<label>.log; the JSON line's ms_per_step is printed.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?tag}
mkdir -p gpurun_out/$TAG
while IFS='|' read -r label envs args; do
  [ -z "$label" ] && continue
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline $args > gpurun_out/$TAG/ab_$label.log 2>&1
  rc=$?
  ms=$(grep '^{' gpurun_out/$TAG/ab_$label.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels_us_per_step',{}); print(d['ms_per_step'], {x:k[x] for x in ('merge_unique','data_blocks','partition_unique','assemble','merge') if x in k})" 2>/dev/null)
  echo "$label rc=$rc ms=$ms"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
