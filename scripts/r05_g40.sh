# round 5 GPU call 40: the derived view reused across calls over the same dataset and spec
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/g40
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_derivatives.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  echo "value-only: $(SRHIP_GRAD_VALUE_ONLY=1 timeout -k 10 120 python -u scripts/grad_bench.py 20 2>&1 | tail -1)"
  echo "gradient:   $(timeout -k 10 120 python -u scripts/grad_bench.py 20 2>&1 | tail -1)"
done | tee $O/grad_bench.log
