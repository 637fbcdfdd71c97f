#!/bin/bash
# The -m gpu suite, then kernel traces of the C2 bench (scripts/trace_ab.sh, BUILDS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
[ -z "${BUILDS:-}" ] || bash scripts/trace_ab.sh
