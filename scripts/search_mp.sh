#!/bin/bash
# C1 / C3 searches with islands in worker processes (:multiprocessing) vs threads, and the device
# search tests; every GPU step under its own time limit, stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/search
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -v --timeout 240 --timeout-method thread > gpurun_out/search/tests.log 2>&1
rc=$?; echo "search tests rc=$rc"; grep -E "PASS|FAIL|passed|failed" gpurun_out/search/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
for cfg in c1 c3; do
  timeout -k 10 300 python -u bench.py --config $cfg --parallelism multiprocessing ${BENCH_EXTRA:-} > gpurun_out/search/${cfg}_mp.json 2> gpurun_out/search/${cfg}_mp.err
  rc=$?; echo "$cfg mp rc=$rc"; tail -c 700 gpurun_out/search/${cfg}_mp.json; echo
  [ $rc -eq 0 ] || exit $rc
done
