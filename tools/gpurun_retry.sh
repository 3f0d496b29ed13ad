#!/bin/bash
# gpurun with retries on INFRASTRUCTURE failures only (no box / box lost while being prepared:
# nothing of the command ran). A command that ran and failed is never retried.
# usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
log=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then sleep 180; continue; fi
  exit $rc
done
exit $rc
