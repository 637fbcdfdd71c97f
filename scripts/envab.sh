#!/bin/bash
# Same-box A/B of environment settings on one build: ENVS="A=1 B=2;A=0" (';' separates settings), REPS runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/envab
export TMPDIR=/tmp
IFS=';' read -ra SETS <<< "${ENVS}"
for rep in $(seq 1 ${REPS:-3}); do
  i=0
  for e in "${SETS[@]}"; do
    i=$((i+1))
    env $e timeout -k 10 200 python -u bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-3} --no-cpu ${BENCH_ARGS:-} > gpurun_out/envab/$i.$rep.json 2> gpurun_out/envab/$i.$rep.err
    rc=$?
    echo "[$e] rep=$rep rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/envab/$i.$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; x=d.get('extra',{}); print('value=%.4f kernel_ms=%.4f no_ee=%.4f derived=%.4f ms_step=%.3f' % (d['value'], r['kernel_ms'], x.get('no_early_exit',{}).get('kernel_ms',0), x.get('derived_columns',{}).get('kernel_ms',0), d.get('ms_per_step', float('nan'))))" 2>&1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
