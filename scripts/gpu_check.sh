#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel-trace profile.
# Stops at the first GPU fault / timeout (no further GPU step after a failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -lt 0 ]; }   # timeouts, kills, aborts, segfaults
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/gpu_tests.log | tail -20
bad $rc && exit $rc
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --headline-only > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof.log
fi
exit 0
