#!/bin/bash
# A/B over (build dir, environment) pairs: COMBOS="build:- build_w12:SRHIP_NO_WIDE=1,X=Y ..."
# runs the bench (no CPU baseline) once per pair against that build's libsrhip.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for c in ${COMBOS:-build:-}; do
  i=$((i + 1))
  b=${c%%:*}
  e=${c#*:}
  envs=()
  [ "$e" = "-" ] || IFS=',' read -ra envs <<< "$e"
  env "${envs[@]}" SRHIP_LIB=$PWD/symbolicregression.jl_amd/$b/libsrhip.so timeout -k 10 200 \
    python -u bench.py --steps 10 --warmup 3 --no-cpu "$@" > gpurun_out/abenv_$i.log 2>&1
  rc=$?
  echo "[$c] rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/abenv_$i.log').read().strip().splitlines()[-1]); print('kernel_ms=%.3f ms_per_step=%.3f' % (d['roofline']['kernel_ms'], d['ms_per_step']))" 2>&1 | tail -1)"
  [ $rc -eq 0 ] || exit $rc
done
