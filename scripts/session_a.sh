#!/bin/bash
# Optimiser GPU tests (incl. the value-only early exit), then the C4 diagnostics.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "optim or c4" > gpurun_out/optim_tests.log 2>&1
rc=$?; echo "optim tests rc=$rc"; tail -3 gpurun_out/optim_tests.log
[ $rc -eq 0 ] || exit $rc
SPLITS="1 3" NO_TRACE=1 bash scripts/c4_diag.sh || exit $?
