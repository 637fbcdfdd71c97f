#!/bin/bash
# PMC passes over scripts/grad_bench.py (the C4 full-population gradient launch), one rocprofv3
# --pmc pass per counter group under its own hard timeout; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${PMCG_DIR:-gpurun_out/pmcg}; mkdir -p $D
export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  echo "pass $i: $counters"
  timeout -s KILL 120 rocprofv3 --pmc $counters -d $D/p$i -o p$i --output-format csv -- python3 scripts/grad_bench.py 5 > $D/p$i.log 2>&1
  rc=$?
  echo "  rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done <<LIST
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM GRBM_GUI_ACTIVE
SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64
FETCH_SIZE GRBM_GUI_ACTIVE
WRITE_SIZE GRBM_GUI_ACTIVE
LIST
