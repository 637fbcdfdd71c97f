# round 5 GPU call 23: C2 scratch -- the setup spill of the lane offset (opaque lane id) and the 64-byte
# spill on the unchecked cos/sin dispatch path (SRHIP_COS_NC=0 build) -- parity, writes, time
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05/scr
mkdir -p $O
L=symbolicregression.jl_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_persistent.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu -k "not c4 and not optim" > $O/tests_new.log 2>&1 || { tail -30 $O/tests_new.log; exit 1; }
tail -1 $O/tests_new.log
SRHIP_LIB=$L/build_nonc/libsrhip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu -k "not c4 and not optim" > $O/tests_nonc.log 2>&1 || { tail -30 $O/tests_nonc.log; exit 1; }
tail -1 $O/tests_nonc.log
i=0
for lib in build_old build build_nonc; do
  i=$((i+1))
  rm -rf gpurun_out/pmc
  SRHIP_LIB=$L/$lib/libsrhip.so PMC_LIST="WRITE_SIZE GRBM_GUI_ACTIVE" BENCH_ARGS="--steps 4 --warmup 2 --no-cpu --headline-only" bash scripts/pmc.sh > $O/pmc_$lib.log 2>&1 || exit $?
  python3 scripts/pmc_step.py gpurun_out/pmc 8 --json $O/pmc_$lib.json > /dev/null || exit $?
  python3 -c "import json; d=json.load(open('$O/pmc_$lib.json')); [print('$lib', '%.3f MB write per evaluation' % (v.get('hbm_write_bytes',0)/1e6)) for k,v in d.items()]"
done
rm -rf gpurun_out/envab
ENVS="SRHIP_LIB=$L/build_old/libsrhip.so;SRHIP_LIB=$L/build/libsrhip.so;SRHIP_LIB=$L/build_nonc/libsrhip.so" REPS=3 BENCH_ARGS="--headline-only --warmup 30" bash scripts/envab.sh > $O/envab.log 2>&1
rc=$?
cat $O/envab.log
exit $rc
