#!/bin/bash
# C4 optimiser diagnostics: launch counts / host vs device time (SRHIP_OPTIM_TIMING=2) with the
# population split over 1 and 3 contexts, then a kernel trace of the split-1 run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c4diag
export TMPDIR=/tmp
for g in ${SPLITS:-1 3}; do
  SRHIP_OPTIM_TIMING=2 SRHIP_OPTIM_SPLIT=$g timeout -k 10 300 python3 -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu \
    > gpurun_out/c4diag/split$g.json 2> gpurun_out/c4diag/split$g.err
  rc=$?; echo "split $g rc=$rc"; grep "srhip optim" gpurun_out/c4diag/split$g.err | tail -4
  python3 -c "import json; d=json.loads(open('gpurun_out/c4diag/split$g.json').read().strip().splitlines()[-1]); print('value', d['value'])"
  [ $rc -eq 0 ] || exit $rc
done
if [ -z "${NO_TRACE:-}" ]; then
  SRHIP_OPTIM_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c4diag/trace -o run --output-format csv -- \
    python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu > gpurun_out/c4diag/trace.log 2>&1
  rc=$?; echo "trace rc=$rc"
fi
