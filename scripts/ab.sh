#!/bin/bash
# A/B: GPU parity tests on the default build, then the bench against each listed build dir.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for b in ${BUILDS:-build}; do
  for rep in 1 2; do
    SRHIP_LIB=$PWD/symbolicregression.jl_amd/$b/libsrhip.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_$b.log 2>&1
    rc=$?
    echo "$b rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$b.log').read().strip().splitlines()[-1]); print('kernel_ms=%.3f ms_per_step=%.3f frac=%.4f' % (d['roofline']['kernel_ms'], d['ms_per_step'], d['roofline']['frac']))" 2>&1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
