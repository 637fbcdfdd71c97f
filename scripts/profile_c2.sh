#!/bin/bash
# C2 profile for profiles/: a rocprofv3 kernel trace (per-dispatch timestamps + stats) of the
# headline bench, then the PMC counter passes (scripts/pmc.sh), each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/trace_c2 gpurun_out/pmc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_c2 -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu --headline-only > gpurun_out/trace_c2.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 gpurun_out/trace_c2.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
[ -n "${NO_PMC:-}" ] || bash scripts/pmc.sh
