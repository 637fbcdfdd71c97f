#!/bin/bash
# Every config's bench line (C2 headline, C4, C1, C3) into gpurun_out/bench_<cfg>.json; stops at the
# first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${CONFIGS:-c2 c4 c1 c3}; do
  timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py --config $cfg ${BENCH_ARGS:-} > gpurun_out/bench_$cfg.log 2>&1
  rc=$?
  echo "$cfg rc=$rc"
  tail -1 gpurun_out/bench_$cfg.log > gpurun_out/bench_$cfg.json
  head -c 600 gpurun_out/bench_$cfg.json; echo
  [ $rc -eq 0 ] || exit $rc
done
