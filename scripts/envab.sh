#!/bin/bash
# A/B over environment settings of one build: the bench once per "NAME=VALUE[,NAME=VALUE]" in ENVS
# ("-" = defaults).  usage: ENVS="- SRHIP_NO_DERIVE=1" scripts/envab.sh [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for e in ${ENVS:--}; do
  i=$((i + 1))
  envs=()
  [ "$e" = "-" ] || IFS=',' read -ra envs <<< "$e"
  env "${envs[@]}" timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu "$@" > gpurun_out/envab_$i.log 2>&1
  rc=$?
  echo "[$e] rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/envab_$i.log').read().strip().splitlines()[-1]); print('kernel_ms=%.3f ms_per_step=%.3f frac=%.4f' % (d['roofline']['kernel_ms'], d['ms_per_step'], d['roofline']['frac']))" 2>&1)"
  [ $rc -eq 0 ] || exit $rc
done
