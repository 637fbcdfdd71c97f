# round 5 GPU call 14: C4 speculation limits A/B (slots, depth per tree, active-tree threshold), same box
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
rm -rf gpurun_out/envab
ENVS="SRHIP_OPTIM_SPEC=32;SRHIP_OPTIM_SPEC=64;SRHIP_OPTIM_SPEC=128 SRHIP_OPTIM_SPEC_DEPTH=128;SRHIP_OPTIM_SPEC=128 SRHIP_OPTIM_SPEC_ACTIVE=128;SRHIP_OPTIM_SPEC=256 SRHIP_OPTIM_SPEC_DEPTH=128 SRHIP_OPTIM_SPEC_ACTIVE=128" REPS=2 STEPS=5 WARMUP=2 BENCH_ARGS="--config c4" bash scripts/envab.sh > gpurun_out/r05/envab_g14.log 2>&1
rc=$?
cat gpurun_out/r05/envab_g14.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/r05/c2_g14_$r.json 2> gpurun_out/r05/c2_g14_$r.err || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/r05/c2_g14_$r.json').read().strip().splitlines()[-1]); pp=d['extra']['population_pipeline']; print(d['ms_per_step'], d['roofline']['kernel_ms'], {k: pp[k] for k in pp if k.endswith('ms') or k.endswith('population')})"
done
