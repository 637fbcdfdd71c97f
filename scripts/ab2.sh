#!/bin/bash
# Same-box A/B of library builds (SRHIP_LIB), interleaved: BUILDS="path1 path2", REPS runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-3}); do
  for b in ${BUILDS}; do
    tag=$(echo $b | tr '/' '_')
    SRHIP_LIB=$PWD/$b/libsrhip.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab/$tag.$rep.json 2> gpurun_out/ab/$tag.$rep.err
    rc=$?
    echo "$b rep=$rep rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/$tag.$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; x=d.get('extra',{}); print('kernel_ms=%.4f no_ee=%.4f derived=%.4f ms_step=%.3f' % (r['kernel_ms'], x.get('no_early_exit',{}).get('kernel_ms',0), x.get('derived_columns',{}).get('kernel_ms',0), d['ms_per_step']))" 2>&1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
