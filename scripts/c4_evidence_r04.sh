#!/bin/bash
# Round-4 C4 evidence after the gradient-kernel changes, on the committed build: GPU suite, smoke, C4
# bench (all-core CPU baseline), gradient + value-only PMC, the split-3 optimiser timing.  Each step
# under its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/c4ev; mkdir -p $F
export TMPDIR=/tmp
step() { echo "== $1"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -30 $F/gpu_tests.log; exit 1; }
tail -1 $F/gpu_tests.log
step smoke
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || exit $?
tail -1 $F/smoke.log
step c4
timeout -k 10 600 python -u bench.py --config c4 > $F/bench_c4.log 2>&1 || exit $?
tail -1 $F/bench_c4.log > $F/bench_c4.json
step grad_bench
timeout -k 10 120 python3 scripts/grad_bench.py 20 > $F/grad_bench.log 2>&1 || exit $?
SRHIP_GRAD_VALUE_ONLY=1 timeout -k 10 120 python3 scripts/grad_bench.py 20 >> $F/grad_bench.log 2>&1 || exit $?
cat $F/grad_bench.log
step pmc_grad
rm -rf gpurun_out/pmcg; bash scripts/pmc_grad.sh > $F/pmc_grad.log 2>&1 || exit $?
python3 scripts/pmc_step.py gpurun_out/pmcg 8 grad_kernel --json $F/pmc_grad_c4.json > /dev/null
step pmc_value_only
rm -rf gpurun_out/pmcv; (export SRHIP_GRAD_VALUE_ONLY=1; PMCG_DIR=gpurun_out/pmcv bash scripts/pmc_grad.sh) > $F/pmc_value.log 2>&1 || exit $?
python3 scripts/pmc_step.py gpurun_out/pmcv 8 grad_kernel --json $F/pmc_value_c4.json > /dev/null
step c4_diag
SPLITS=3 NO_TRACE=1 bash scripts/c4_diag.sh > $F/c4_diag.log 2>&1 || exit $?
cat $F/c4_diag.log
echo done
