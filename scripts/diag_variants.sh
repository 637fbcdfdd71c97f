#!/bin/bash
# Runs the step-by-step ABI driver against compiler-flag variants of libsrhip.so.
# Stops at the first timeout / crash (no further GPU step after a failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in build_c build_b build; do
  echo "== variant $v" | tee -a gpurun_out/diag.log
  LD_LIBRARY_PATH=$PWD/symbolicregression.jl_amd/$v timeout -k 5 45 tools/build/srhip_diag >> gpurun_out/diag.log 2>&1
  rc=$?
  echo "rc=$rc" | tee -a gpurun_out/diag.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
