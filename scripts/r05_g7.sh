# round 5 GPU call 7: same-box A/B of builds -- Julia trig bodies interleaving 1 / 2 / 4 rows (SRHIP_TRIG_ILP)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
rm -rf gpurun_out/envab
L=symbolicregression.jl_amd
ENVS="SRHIP_LIB=$L/build/libsrhip.so;SRHIP_LIB=$L/build_ilp2/libsrhip.so;SRHIP_LIB=$L/build_ilp4/libsrhip.so" REPS=3 BENCH_ARGS="--headline-only --warmup 30" bash scripts/envab.sh > gpurun_out/r05/envab_g7.log 2>&1
rc=$?
cp -r gpurun_out/envab gpurun_out/r05/envab_g7
exit $rc
