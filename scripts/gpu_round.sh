#!/bin/bash
# Round-4 GPU session: the -m gpu suite, the rowshard bench (native RCCL at world 1), then a same-box
# A/B of library builds on the C2 bench (BUILDS, REPS).  Each step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest -m gpu rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -20
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
if [ -n "${ROWSHARD:-}" ]; then
  timeout -k 10 300 python -u bench.py --mode rowshard --steps 10 --warmup 5 > gpurun_out/rowshard_n1.log 2>&1
  rc=$?; echo "rowshard rc=$rc"; tail -1 gpurun_out/rowshard_n1.log | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${BUILDS:-}" ]; then bash scripts/ab2.sh || exit $?; fi
# BENCHES="c4:--config c4 --no-cpu;c2:": extra bench lines, name:args separated by ';'
if [ -n "${BENCHES:-}" ]; then
  IFS=';' read -ra items <<< "$BENCHES"
  for it in "${items[@]}"; do
    nm=${it%%:*}; args=${it#*:}
    timeout -k 10 400 python -u bench.py $args > gpurun_out/bench_$nm.json 2> gpurun_out/bench_$nm.err
    rc=$?; echo "bench $nm rc=$rc"; tail -1 gpurun_out/bench_$nm.json | cut -c1-400
    [ $rc -eq 0 ] || exit $rc
  done
fi
