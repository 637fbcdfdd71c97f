# round 5 GPU call 20: C4 optimiser split (host threads / contexts) re-measured on the round-5 build
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
rm -rf gpurun_out/envab
ENVS="SRHIP_OPTIM_SPLIT=3;SRHIP_OPTIM_SPLIT=2;SRHIP_OPTIM_SPLIT=4;SRHIP_OPTIM_SPLIT=3 SRHIP_OPTIM_SPEC=16" REPS=2 STEPS=5 WARMUP=2 BENCH_ARGS="--config c4" bash scripts/envab.sh > gpurun_out/r05/envab_g20.log 2>&1
rc=$?
cat gpurun_out/r05/envab_g20.log
exit $rc
