#!/bin/bash
# Round-end evidence on the committed build: GPU suite, smoke, C2 bench (with CPU baseline), the
# headline-only kernel trace, PMC passes, then C4 / C1 / C3 bench lines.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -1 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu --headline-only > gpurun_out/prof.log 2>&1 || exit $?
scripts/pmc.sh > gpurun_out/pmc.log 2>&1 || exit $?
CONFIGS="c2 c4 c1 c3" scripts/bench_all.sh
