# round 5 GPU call 39: C4 evidence on the final gradient-program build (binary uniform forms included):
# C4 bench with its CPU baseline, gradient PMC passes, the per-group diagnosis, a C4 kernel trace
set -u
cd $GRAFT_REPO_ROOT
F=gpurun_out/final5c4
mkdir -p $F
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --config c4 > $F/bench_c4.log 2>&1 || exit $?
tail -1 $F/bench_c4.log > $F/bench_c4.json
rm -rf gpurun_out/pmcg; bash scripts/pmc_grad.sh > $F/pmc_grad.log 2>&1 || exit $?
python3 scripts/pmc_step.py gpurun_out/pmcg 8 grad_kernel --json $F/pmc_grad_c4.json > /dev/null
SPLITS=3 NO_TRACE=1 bash scripts/c4_diag.sh > $F/c4_diag.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d $F/c4trace -o run --output-format csv -- python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu > $F/c4trace.log 2>&1 || exit $?
python3 scripts/c4_trace.py $F/c4trace/run_kernel_trace.csv --json $F/c4_trace.json > /dev/null || exit $?
python3 -c "
import json; d=json.loads(open('$F/bench_c4.json').read()); print('c4', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['cpu_baseline']['value'])"
echo done
