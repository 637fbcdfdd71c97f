#!/bin/bash
# A/B of build dirs on several operator mixes (bench kernel time only; no tests).
# usage: BUILDS="build build_x" MIXES="+,-,*,/:cos,exp +,-,*:" bash scripts/abmix.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in ${BUILDS:-build}; do
  for mix in ${MIXES:-+,-,*,/:cos,exp +,-,*:}; do
    bo=${mix%%:*}; u=${mix##*:}
    SRHIP_LIB=$PWD/symbolicregression.jl_amd/$b/libsrhip.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --binops "$bo" --unaops "$u" > gpurun_out/abmix.log 2>&1
    rc=$?
    echo "$b [$bo] [$u] rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/abmix.log').read().strip().splitlines()[-1]); print('kernel_ms=%.3f ms_per_step=%.3f' % (d['roofline']['kernel_ms'], d['ms_per_step']))" 2>&1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
