# round 5 GPU call 37: gradient programs evaluate unary operators of constant subtrees once per lane
# (UN_UNIFORM_FLAG): gradient / value-only launches and C4 against SRHIP_GRAD_UNIFORM=0, then the
# gradient and optimiser GPU tests
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/g37
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py -x -q --timeout 300 --timeout-method thread -m gpu -k "uniform or derived or split or speculative" > $O/tests0.log 2>&1 || { tail -30 $O/tests0.log; exit 1; }
tail -1 $O/tests0.log
for rep in 1 2; do
  for u in 0 1; do
    echo "uniform=$u value-only: $(SRHIP_GRAD_UNIFORM=$u SRHIP_GRAD_VALUE_ONLY=1 timeout -k 10 120 python -u scripts/grad_bench.py 20 2>&1 | tail -1)"
    echo "uniform=$u gradient:   $(SRHIP_GRAD_UNIFORM=$u timeout -k 10 120 python -u scripts/grad_bench.py 20 2>&1 | tail -1)"
  done
done
rm -rf gpurun_out/envab
ENVS="SRHIP_GRAD_UNIFORM=0;SRHIP_GRAD_UNIFORM=1" REPS=3 STEPS=5 WARMUP=2 BENCH_ARGS="--config c4" bash scripts/envab.sh > $O/envab.log 2>&1
rc=$?
cat $O/envab.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_derivatives.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
