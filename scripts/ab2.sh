#!/bin/bash
# Same-box A/B of library builds (SRHIP_LIB), interleaved: BUILDS="path1 path2[:ENV=V[,ENV2=V2]]", REPS
# runs each; an entry's optional ":ENV=V,..." suffix sets environment variables for its runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-3}); do
  for spec in ${BUILDS}; do
    b=${spec%%:*}
    envs=""
    [ "$spec" != "$b" ] && envs=$(echo "${spec#*:}" | tr ',' ' ')
    tag=$(echo "$spec" | tr '/:=,' '____')
    env $envs SRHIP_LIB=$PWD/$b/libsrhip.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab/$tag.$rep.json 2> gpurun_out/ab/$tag.$rep.err
    rc=$?
    echo "$spec rep=$rep rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/$tag.$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; x=d.get('extra',{}); print('kernel_ms=%.4f ms_step=%.3f undecided=%s' % (r['kernel_ms'], d['ms_per_step'], x.get('undecided_trees_per_step')))" 2>&1 | tail -1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
