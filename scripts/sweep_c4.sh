#!/bin/bash
# C4 optimiser-parameter sweep on one box: each setting one bench run, each under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep4
export TMPDIR=/tmp
for s in ${SETTINGS:-"base:"}; do
  name=${s%%:*}; envs=${s#*:}
  env $envs timeout -k 10 300 python3 -u bench.py --config c4 --no-cpu > gpurun_out/sweep4/$name.log 2>&1 || exit $?
  echo "$name $envs $(python3 -c "import json; d=json.loads(open('gpurun_out/sweep4/$name.log').read().strip().splitlines()[-1]); print('ms=%.1f improved=%d med=%.6g' % (d['value'], d['improved_trees'], d['median_loss_after']))")"
done
