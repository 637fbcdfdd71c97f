# round 5 GPU call 11: where C2's HBM writes come from -- WRITE_SIZE / FETCH_SIZE per step against the
# population size (partials scale with trees x row blocks; a per-wave constant is the intercept)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05/wsz
mkdir -p $O
for nt in 1024 256 64 16; do
  rm -rf gpurun_out/pmc
  PMC_LIST="WRITE_SIZE GRBM_GUI_ACTIVE
FETCH_SIZE GRBM_GUI_ACTIVE" BENCH_ARGS="--steps 4 --warmup 2 --no-cpu --headline-only --ntrees $nt" bash scripts/pmc.sh > $O/pmc_$nt.log 2>&1 || exit $?
  python3 scripts/pmc_step.py gpurun_out/pmc 4 --json $O/pmc_$nt.json > /dev/null || exit $?
  python3 scripts/pmc_step.py gpurun_out/pmc 4 reduce --json $O/pmc_reduce_$nt.json > /dev/null || exit $?
  python3 -c "import json; d=json.load(open('$O/pmc_$nt.json')); [print($nt, k[:50], '%.3f MB write %.3f MB fetch' % (v.get('hbm_write_bytes',0)/1e6, v.get('hbm_fetch_bytes',0)/1e6)) for k,v in d.items()]"
done
