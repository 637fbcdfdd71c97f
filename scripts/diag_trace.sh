#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for stop in 0; do
  echo "== SRHIP_DEBUG_STOP=$stop" >> gpurun_out/diag.log
  SRHIP_DEBUG_STOP=$stop SRHIP_TRACE=1 timeout -k 5 20 tools/build/srhip_diag >> gpurun_out/diag.log 2>&1
  rc=$?
  echo "rc=$rc" | tee -a gpurun_out/diag.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
