# round 5 GPU call 6: C2 launch-shape A/B with Julia's trig (probe blocks, row-block rows), same box
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
rm -rf gpurun_out/envab
ENVS="SRHIP_PROBE_BLOCKS=4;SRHIP_PROBE_BLOCKS=2;SRHIP_PROBE_BLOCKS=6;SRHIP_PRB_ROWS=1024;SRHIP_PRB_ROWS=4096;SRHIP_PROBE_BLOCKS=4" REPS=2 BENCH_ARGS="--headline-only --warmup 30" bash scripts/envab.sh > gpurun_out/r05/envab_g6.log 2>&1
rc=$?
cp -r gpurun_out/envab gpurun_out/r05/envab_g6
exit $rc
