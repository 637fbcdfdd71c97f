#!/bin/bash
# Same-box A/B of environment settings on the fresh-population pipeline section of the C2 bench:
# ENVS="A=1;B=2" (';' separates settings; an empty entry = defaults), REPS runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pipeab
export TMPDIR=/tmp
IFS=';' read -ra SETS <<< "${ENVS}"
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for e in "${SETS[@]}"; do
    i=$((i+1))
    env $e timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/pipeab/$i.$rep.json 2> gpurun_out/pipeab/$i.$rep.err
    rc=$?
    echo "[$e] rep=$rep rc=$rc $(python3 -c "
import json; d=json.loads(open('gpurun_out/pipeab/$i.$rep.json').read().strip().splitlines()[-1]); p=d['extra']['population_pipeline']
print('pipe %.4f kern %.4f over %.4f seq %.4f two %.4f compile %.4f iters %s' % (p['pipelined_ms_per_population'], p['pipelined_kernel_ms'], p['pipelined_over_kernel_ms'], p['sequential_ms_per_population'], p['two_stream_ms_per_population'], p['compile_ms_fresh'], p['pipelined_phases_ms']['iterations']))" 2>&1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
