# round 5 GPU call 25: gradient-record folding in the workgroup -- optimiser suites (bitwise), the
# gradient / value-only launches with and without folding (time, checksum, HBM writes), C4 A/B
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05/fold
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_configs.py tests/test_gpu_derivatives.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for f in 0 64; do
  echo "fold_min $f value-only: $(SRHIP_GRAD_FOLD_MIN=$f SRHIP_GRAD_VALUE_ONLY=1 timeout -k 10 120 python -u scripts/grad_bench.py 20 2>&1 | tail -1)"
  echo "fold_min $f gradient:   $(SRHIP_GRAD_FOLD_MIN=$f timeout -k 10 120 python -u scripts/grad_bench.py 20 2>&1 | tail -1)"
  rm -rf gpurun_out/pmcw
  for c in "WRITE_SIZE GRBM_GUI_ACTIVE" "FETCH_SIZE GRBM_GUI_ACTIVE"; do
    SRHIP_GRAD_FOLD_MIN=$f timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmcw/$(echo $c | cut -d' ' -f1) -o p --output-format csv -- python3 scripts/grad_bench.py 5 > $O/pmcw_$f.log 2>&1 || exit $?
  done
  python3 scripts/pmc_step.py gpurun_out/pmcw 8 grad_kernel --json $O/pmc_grad_fold$f.json > /dev/null || exit $?
  python3 -c "import json; d=json.load(open('$O/pmc_grad_fold$f.json')); [print('fold_min $f', k[:48], '%.2f MB write %.2f MB fetch per launch' % (v.get('hbm_write_bytes',0)/1e6, v.get('hbm_fetch_bytes',0)/1e6)) for k,v in d.items()]"
done
rm -rf gpurun_out/envab
ENVS="SRHIP_GRAD_FOLD_MIN=0;SRHIP_GRAD_FOLD_MIN=64;SRHIP_GRAD_FOLD_MIN=16" REPS=2 STEPS=5 WARMUP=2 BENCH_ARGS="--config c4" bash scripts/envab.sh > $O/envab.log 2>&1
rc=$?
cat $O/envab.log
exit $rc
