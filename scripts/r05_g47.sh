# round 5 GPU call 47: tangent-uniform operators in gradient launches: exactness tests, gradient /
# value-only launches against the previous build (build_prev) on the same box, C4 A/B
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/g47
mkdir -p $O
export TMPDIR=/tmp
L=symbolicregression.jl_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_derivatives.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for lib in build_prev build; do
    echo "$lib value-only: $(SRHIP_LIB=$L/$lib/libsrhip.so SRHIP_GRAD_VALUE_ONLY=1 timeout -k 10 120 python -u scripts/grad_bench.py 20 2>&1 | tail -1)"
    echo "$lib gradient:   $(SRHIP_LIB=$L/$lib/libsrhip.so timeout -k 10 120 python -u scripts/grad_bench.py 20 2>&1 | tail -1)"
  done
done | tee $O/grad_bench.log
rm -rf gpurun_out/envab
ENVS="SRHIP_LIB=$L/build_prev/libsrhip.so;SRHIP_LIB=$L/build/libsrhip.so" REPS=3 STEPS=5 WARMUP=2 BENCH_ARGS="--config c4" bash scripts/envab.sh > $O/envab.log 2>&1
rc=$?
cat $O/envab.log
exit $rc
