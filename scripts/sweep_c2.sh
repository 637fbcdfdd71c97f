#!/bin/bash
# C2 launch-parameter sweep on one box: each setting one bench run (headline only), each under its
# own time limit; prints kernel ms per setting.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
for s in ${SETTINGS:-"base:"}; do
  name=${s%%:*}; envs=${s#*:}
  env $envs timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 30 --no-cpu --headline-only > gpurun_out/sweep/$name.log 2>&1 || exit $?
  echo "$name $envs $(python3 -c "import json; d=json.loads(open('gpurun_out/sweep/$name.log').read().strip().splitlines()[-1]); print('kernel_ms=%.4f value=%.4g' % (d['roofline']['kernel_ms'], d['value']))")"
done
