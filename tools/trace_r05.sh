#!/bin/bash
# Kernel traces of bench configs (round 5 chain-server diagnosis): one
# rocprofv3 --kernel-trace --stats run per "name|ENV=..|args" spec in RUNS.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05t}
mkdir -p $OUT
IFS=';' read -ra SPECS <<< "$RUNS"
for spec in "${SPECS[@]}"; do
  [ -z "$spec" ] && continue
  IFS='|' read -r name envs args <<< "$spec"
  for kv in $envs; do export "$kv"; done
  timeout -k 10 ${LIMIT:-240} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o run -- python3 -u bench.py $args > $OUT/$name.log 2>&1
  rc=$?
  for kv in $envs; do unset "${kv%%=*}"; done
  echo "== $name rc=$rc $(tail -1 $OUT/$name.log | cut -c1-160)"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
echo TRACE_DONE
