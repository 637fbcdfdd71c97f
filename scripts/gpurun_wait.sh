#!/bin/bash
# gpurun, re-submitted only while the pool reports no free slot (exit 3: nothing ran, nothing charged);
# any other outcome (success, a failure, a refusal) is returned as is.  usage: gpurun_wait.sh TIMEOUT 'cmd'
t=$1; shift
for i in $(seq 1 15); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_wait] no slot (try $i); retrying in 120 s"
  sleep 120
done
exit 3
