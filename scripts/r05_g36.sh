# round 5 GPU call 36: gradient programs read heavy operators of features from a derived view:
# exactness tests first, then gradient / value-only launches and C4 against SRHIP_GRAD_DERIVED=0
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/g36
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_derivatives.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for d in 0 1; do
    echo "derived=$d value-only: $(SRHIP_GRAD_DERIVED=$d SRHIP_GRAD_VALUE_ONLY=1 timeout -k 10 120 python -u scripts/grad_bench.py 20 2>&1 | tail -1)"
    echo "derived=$d gradient:   $(SRHIP_GRAD_DERIVED=$d timeout -k 10 120 python -u scripts/grad_bench.py 20 2>&1 | tail -1)"
  done
done | tee $O/grad_bench.log
rm -rf gpurun_out/envab
ENVS="SRHIP_GRAD_DERIVED=0;SRHIP_GRAD_DERIVED=1" REPS=3 STEPS=5 WARMUP=2 BENCH_ARGS="--config c4" bash scripts/envab.sh > $O/envab.log 2>&1
rc=$?
cat $O/envab.log
exit $rc
