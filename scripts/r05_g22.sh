# round 5 GPU call 22: calls 21 (value-only rows A/B) and 20 (optimiser split) in one session
# suites on the new build, then value-only pass and C4 A/B against the previous build
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05
mkdir -p $O
L=symbolicregression.jl_amd
timeout -k 10 900 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_configs.py tests/test_gpu_derivatives.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/g21_tests.log 2>&1 || { tail -30 $O/g21_tests.log; exit 1; }
tail -1 $O/g21_tests.log
for rep in 1 2; do
  for lib in build_old build; do
    echo "$lib value-only: $(SRHIP_LIB=$L/$lib/libsrhip.so SRHIP_GRAD_VALUE_ONLY=1 timeout -k 10 120 python -u scripts/grad_bench.py 20 2>&1 | tail -1)"
    echo "$lib gradient:   $(SRHIP_LIB=$L/$lib/libsrhip.so timeout -k 10 120 python -u scripts/grad_bench.py 20 2>&1 | tail -1)"
  done
done
rm -rf gpurun_out/envab
ENVS="SRHIP_LIB=$L/build_old/libsrhip.so;SRHIP_LIB=$L/build/libsrhip.so" REPS=3 STEPS=5 WARMUP=2 BENCH_ARGS="--config c4" bash scripts/envab.sh > $O/envab_g21.log 2>&1
rc=$?
cat $O/envab_g21.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/envab
ENVS="SRHIP_OPTIM_SPLIT=3;SRHIP_OPTIM_SPLIT=2;SRHIP_OPTIM_SPLIT=4;SRHIP_OPTIM_SPLIT=3 SRHIP_OPTIM_SPEC=16" REPS=2 STEPS=5 WARMUP=2 BENCH_ARGS="--config c4" bash scripts/envab.sh > gpurun_out/r05/envab_g20.log 2>&1
rc=$?
cat gpurun_out/r05/envab_g20.log
exit $rc
