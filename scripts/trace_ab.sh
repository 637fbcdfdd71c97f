#!/bin/bash
# Kernel traces of the C2 bench for several library builds / environments (BUILDS as in ab2.sh:
# "path[:ENV=V,...]"), one rocprofv3 --kernel-trace run each, for per-dispatch timelines
# (scripts/step_timeline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tab
export TMPDIR=/tmp
for spec in ${BUILDS}; do
  b=${spec%%:*}
  envs=""
  [ "$spec" != "$b" ] && envs=$(echo "${spec#*:}" | tr ',' ' ')
  tag=$(echo "$spec" | tr '/:=,' '____')
  for kv in $envs; do export "$kv"; done
  SRHIP_LIB=$PWD/$b/libsrhip.so timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tab/$tag -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu --headline-only > gpurun_out/tab/$tag.log 2>&1
  rc=$?
  for kv in $envs; do unset "${kv%%=*}"; done
  echo "$spec rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
