# round 5 GPU call 26: the non-folded gradient path after the folding change against the build before it
# (same box): gradient / value-only launches and C4; then the new fold equality test
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/prefold
mkdir -p $O
L=symbolicregression.jl_amd
for rep in 1 2; do
  for lib in build_prefold build; do
    echo "$lib value-only: $(SRHIP_LIB=$L/$lib/libsrhip.so SRHIP_GRAD_VALUE_ONLY=1 timeout -k 10 120 python -u scripts/grad_bench.py 20 2>&1 | tail -1)"
    echo "$lib gradient:   $(SRHIP_LIB=$L/$lib/libsrhip.so timeout -k 10 120 python -u scripts/grad_bench.py 20 2>&1 | tail -1)"
  done
done
rm -rf gpurun_out/envab
ENVS="SRHIP_LIB=$L/build_prefold/libsrhip.so;SRHIP_LIB=$L/build/libsrhip.so" REPS=3 STEPS=5 WARMUP=2 BENCH_ARGS="--config c4" bash scripts/envab.sh > $O/envab.log 2>&1
rc=$?
cat $O/envab.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py -x -q --timeout 300 --timeout-method thread -m gpu -k "folded or inline or screening" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
