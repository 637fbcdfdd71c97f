# round 5 GPU call 10: value-only screening -- optimiser / C4 GPU tests, then a same-box C4 A/B of
# SRHIP_GRAD_SCREEN (0 = off, 1 = every value-only pass, 16 = passes of >= 16 chunks)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r05/g10_tests.log 2>&1 || { tail -30 gpurun_out/r05/g10_tests.log; exit 1; }
tail -2 gpurun_out/r05/g10_tests.log
rm -rf gpurun_out/envab
ENVS="SRHIP_GRAD_SCREEN=0;SRHIP_GRAD_SCREEN=1;SRHIP_GRAD_SCREEN=16" REPS=3 STEPS=5 WARMUP=2 BENCH_ARGS="--config c4" bash scripts/envab.sh > gpurun_out/r05/envab_g10.log 2>&1
rc=$?
cat gpurun_out/r05/envab_g10.log
cp -r gpurun_out/envab gpurun_out/r05/envab_g10
exit $rc
