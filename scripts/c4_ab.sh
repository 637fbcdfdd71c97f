#!/bin/bash
# Same-box A/B of the C4 bench over environment settings: SPECS="name:ENV=V,ENV2=V2 name2:" (REPS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c4ab
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-2}); do
  for spec in ${SPECS}; do
    nm=${spec%%:*}; envs=$(echo "${spec#*:}" | tr ',' ' ')
    env $envs timeout -k 10 300 python3 -u bench.py --config c4 --steps ${STEPS:-4} --warmup 1 --no-cpu \
      > gpurun_out/c4ab/$nm.$rep.json 2> gpurun_out/c4ab/$nm.$rep.err
    rc=$?
    echo "$nm rep=$rep rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/c4ab/$nm.$rep.json').read().strip().splitlines()[-1]); print('value %.1f ms improved %s' % (d['value'], d.get('improved_trees')))" 2>&1 | tail -1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
