# round 5 GPU call 24: unchecked cos / sin as an operand flag instead of handlers of their own -- full GPU
# suite, then writes and a same-box C2 A/B against the previous build
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05/ncflag
mkdir -p $O
L=symbolicregression.jl_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in build_prev build; do
  rm -rf gpurun_out/pmc
  SRHIP_LIB=$L/$lib/libsrhip.so PMC_LIST="WRITE_SIZE GRBM_GUI_ACTIVE" BENCH_ARGS="--steps 4 --warmup 2 --no-cpu --headline-only" bash scripts/pmc.sh > $O/pmc_$lib.log 2>&1 || exit $?
  python3 scripts/pmc_step.py gpurun_out/pmc 8 --json $O/pmc_$lib.json > /dev/null || exit $?
  python3 -c "import json; d=json.load(open('$O/pmc_$lib.json')); [print('$lib', '%.3f MB write per evaluation' % (v.get('hbm_write_bytes',0)/1e6)) for k,v in d.items()]"
done
rm -rf gpurun_out/envab
ENVS="SRHIP_LIB=$L/build_prev/libsrhip.so;SRHIP_LIB=$L/build/libsrhip.so" REPS=4 BENCH_ARGS="--headline-only --warmup 30" bash scripts/envab.sh > $O/envab.log 2>&1
rc=$?
cat $O/envab.log
exit $rc
