#!/bin/bash
# C4 optimiser A/B over SRHIP_GRAD_RB (gradient row-block size) and SRHIP_OPTIM_SPEC (speculative
# line-search slots), with the optimiser's timing split and launch statistics.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rb in ${RBS:-256}; do
  for spec in ${SPECS:-256}; do
  for vt in ${VTS:-1}; do
    tag=rb${rb}_spec${spec}_vt${vt}
    SRHIP_GRAD_RB=$rb SRHIP_OPTIM_SPEC=$spec SRHIP_OPTIM_VALUE_TRIALS=$vt SRHIP_OPTIM_TIMING=2 timeout -k 10 300 \
      python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/c4_$tag.log 2>&1
    rc=$?
    echo "$tag rc=$rc"
    grep 'srhip optim' gpurun_out/c4_$tag.log | tail -6
    python3 -c "import json; d=json.loads(open('gpurun_out/c4_$tag.log').read().strip().splitlines()[-1]); print('  value_ms=%.1f grad_kernel_ms=%.3f frac=%.4f improved=%d' % (d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['improved_trees']))"
    [ $rc -eq 0 ] || exit $rc
  done
  done
done
