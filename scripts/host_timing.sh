#!/bin/bash
# Host-side split of the C2 step (SRHIP_HOST_TIMING=1: before the wait / in the wait / after it),
# with the spin wait (default) and with SRHIP_SYNC_BLOCK=1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/host
for v in block spin; do
  extra=""; [ $v = spin ] && extra="SRHIP_SYNC_SPIN=1"
  env SRHIP_HOST_TIMING=1 $extra timeout -k 10 200 python3 -u bench.py --steps 100 --warmup 3 --no-cpu --headline-only \
    > gpurun_out/host/$v.json 2> gpurun_out/host/$v.err
  rc=$?; echo "$v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/host/$v.json)"; grep "srhip host" gpurun_out/host/$v.err | tail -2
  [ $rc -eq 0 ] || exit $rc
done
