#!/bin/bash
# GPU tests (PYTEST_K subset), then a same-box A/B of environment settings (ENVS, ';'-separated) and
# one rocprofv3 kernel trace of the headline (gpurun_out/prof).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${PYTEST_K:-}" ]; then bash scripts/gpu_tests.sh || exit $?; fi
REPS=${REPS:-1} BENCH_ARGS=--headline-only bash scripts/envab.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 5 --no-cpu --headline-only > gpurun_out/prof.log 2>&1 || exit $?
python3 scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv
