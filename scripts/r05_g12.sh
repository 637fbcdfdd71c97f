# round 5 GPU call 12: C2 write traffic -- failed-tree marks through device-coherent atomics (default build)
# vs through the XCD's L2 (build_flag, SRHIP_FLAG_CACHED=1): parity suites on the variant, WRITE/FETCH_SIZE
# per evaluation (default, default without early exit, variant), then a same-box timing A/B
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05/flag
mkdir -p $O
L=symbolicregression.jl_amd
SRHIP_LIB=$L/build_flag/libsrhip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_persistent.py tests/test_gpu_precise.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests_flag.log 2>&1 || { tail -30 $O/tests_flag.log; exit 1; }
tail -1 $O/tests_flag.log
i=0
for e in "SRHIP_LIB=$L/build/libsrhip.so" "SRHIP_LIB=$L/build/libsrhip.so SRHIP_NO_EARLY_EXIT=1" "SRHIP_LIB=$L/build_flag/libsrhip.so"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc
  env $e PMC_LIST="WRITE_SIZE GRBM_GUI_ACTIVE
FETCH_SIZE GRBM_GUI_ACTIVE" BENCH_ARGS="--steps 4 --warmup 2 --no-cpu --headline-only" bash scripts/pmc.sh > $O/pmc_$i.log 2>&1 || exit $?
  python3 scripts/pmc_step.py gpurun_out/pmc 8 --json $O/pmc_$i.json > /dev/null || exit $?
  python3 -c "import json; d=json.load(open('$O/pmc_$i.json')); [print('$e', '%.3f MB write %.3f MB fetch per evaluation' % (v.get('hbm_write_bytes',0)/1e6, v.get('hbm_fetch_bytes',0)/1e6)) for k,v in d.items()]"
done
rm -rf gpurun_out/envab
ENVS="SRHIP_LIB=$L/build/libsrhip.so;SRHIP_LIB=$L/build_flag/libsrhip.so" REPS=3 BENCH_ARGS="--headline-only --warmup 30" bash scripts/envab.sh > $O/envab.log 2>&1
rc=$?
cat $O/envab.log
exit $rc
