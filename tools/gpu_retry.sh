#!/bin/bash
# Run one gpurun call, re-queuing only while the pod has no free slot (gpurun's "transient"
# status: nothing ran, nothing was charged).  Any run that started is never repeated.
#   tools/gpu_retry.sh <log> <timeout-s> <command...>
log=$1; to=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  grep -q "status=transient" "$log" || exit $rc
  sleep 90
done
exit $rc
