#!/bin/bash
# Calls gpurun, retrying only while it reports no free slot or box (exit 3: nothing ran, nothing
# charged), every 2 minutes, at most 12 times.  Any other outcome -- success, a failure of the
# command, a refusal -- is returned as is.  usage: tools/gpurun_retry.sh TIMEOUT 'command'
t=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 120
done
exit 3
