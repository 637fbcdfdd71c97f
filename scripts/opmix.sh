#!/bin/bash
# Per-operator cost probe: the C2 bench with different operator sets.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mix in "+,-,*,/:cos,exp" "+,-,*:" "+,-,*,/:" "+,-,*:cos" "+,-,*:exp" "+,-,*:sin,cos"; do
  b=${mix%%:*}; u=${mix##*:}
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu --binops "$b" --unaops "$u" > gpurun_out/mix.log 2>&1
  rc=$?
  echo "[$b] [$u] rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/mix.log').read().strip().splitlines()[-1]); c=d['config']; print('kernel_ms=%.3f nodes=%d ops=%d' % (d['roofline']['kernel_ms'], c['nodes_per_step'], c['opnodes_per_step']))" 2>&1)"
  [ $rc -eq 0 ] || exit $rc
done
