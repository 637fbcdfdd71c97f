#!/bin/bash
# Tuning matrix for the interpreter launch shape: (build dir, SRHIP_RB_ROWS) pairs -> C2 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${CFGS:-build:0}; do
  b=${cfg%%:*}; rb=${cfg##*:}
  SRHIP_RB_ROWS=$rb SRHIP_LIB=$PWD/symbolicregression.jl_amd/$b/libsrhip.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/tune_${b}_${rb}.log 2>&1
  rc=$?
  echo "$b rb=$rb rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/tune_${b}_${rb}.log').read().strip().splitlines()[-1]); print('kernel_ms=%.3f' % d['roofline']['kernel_ms'])" 2>&1)"
  [ $rc -eq 0 ] || exit $rc
done
