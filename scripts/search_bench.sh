#!/bin/bash
# GPU session: parity tests, then the search configs of bench.py (C1, C3) on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for c in ${CONFIGS:-c1 c3}; do
  timeout -k 10 400 python -u bench.py --config $c ${BENCH_ARGS:-} > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; tail -c 1500 gpurun_out/bench_$c.log
  [ $rc -eq 0 ] || exit $rc
done
