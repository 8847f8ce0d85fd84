#!/bin/bash
# Retry a gpurun call only while the pod has no free slot (nothing ran, nothing charged).
LOG=$1; shift  # usage: tools/gpurun_retry.sh LOGFILE <gpurun arguments>
for i in $(seq 1 15); do
  timeout 2700 /usr/local/graft/bin/gpurun "$@" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG; then sleep 90; continue; fi
  break
done
echo "done rc=$rc" >> $LOG
