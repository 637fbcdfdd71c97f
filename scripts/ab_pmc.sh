#!/bin/bash
# Same-box A/B of environment settings (scripts/envab.sh, ENVS="A=1;B=2") followed by one PMC pass per
# setting in PMC_ENVS (';'-separated) over the headline kernel (counters PMC_COUNTERS).  Stops at the
# first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abpmc
export TMPDIR=/tmp
BENCH_ARGS="${BENCH_ARGS:---headline-only}" REPS=${REPS:-1} bash scripts/envab.sh || exit $?
IFS=';' read -ra PSETS <<< "${PMC_ENVS:-}"
i=0
for e in "${PSETS[@]}"; do
  i=$((i+1))
  echo "pmc [$e]"
  env $e timeout -s KILL 120 rocprofv3 --pmc ${PMC_COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE} \
    -d gpurun_out/abpmc/p$i -o p$i --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --headline-only \
    > gpurun_out/abpmc/p$i.log 2>&1
  rc=$?
  echo "  rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
