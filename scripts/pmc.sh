#!/bin/bash
# PMC counter passes over a short bench run (one rocprofv3 --pmc pass per counter group; each
# pass under its own hard timeout; stop at the first failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu --headline-only}
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  echo "pass $i: $counters"
  timeout -s KILL 120 rocprofv3 --pmc $counters -d gpurun_out/pmc/p$i -o p$i --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "  rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done <<LIST
${PMC_LIST:-$(cat <<'DEFAULT'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VMEM GRBM_GUI_ACTIVE
SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE
SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT
FETCH_SIZE GRBM_GUI_ACTIVE
WRITE_SIZE GRBM_GUI_ACTIVE
DEFAULT
)}
LIST
