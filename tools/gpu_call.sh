#!/bin/bash
# gpu_call.sh TIMEOUT 'COMMAND' — one gpurun call; when the pod has no free
# slot (exit 3: nothing ran, nothing charged) wait a minute and ask again, at
# most 15 times.  Any other outcome (success or failure) is final.
t=$1; shift
for i in $(seq 1 15); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 60
done
exit 3
