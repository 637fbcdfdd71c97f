#!/bin/bash
# Per-operator counters (scripts/op_costs.py) in two rocprofv3 --pmc passes, each under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/opc
export TMPDIR=/tmp
timeout -k 10 120 python3 -u scripts/op_costs.py 3 > gpurun_out/opc/plain.log 2>&1 || exit $?
cp gpurun_out/op_costs_order.json gpurun_out/opc/order.json
i=0
for counters in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE" \
                "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $counters -d gpurun_out/opc/p$i -o p$i --output-format csv -- python3 scripts/op_costs.py 2 > gpurun_out/opc/p$i.log 2>&1 || exit $?
done
python3 scripts/op_costs_pmc.py gpurun_out/opc gpurun_out/op_costs_order.json --json gpurun_out/opc/op_costs.json > /dev/null
