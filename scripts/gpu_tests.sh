#!/bin/bash
# The -m gpu suite alone (no -x: every failure is listed), one process, per-test time limits.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest -m gpu rc=$rc"
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -40
exit $rc
