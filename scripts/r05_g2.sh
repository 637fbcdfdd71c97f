# round 5 GPU call 2: the Float32 restart oracle test, C2 after the rematerialised setup addresses,
# its per-step PMC passes, the device-resident row-shard bench
set -u
cd $GRAFT_REPO_ROOT
F=gpurun_out/r05
mkdir -p $F
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "restart_float32" -x -v --timeout 240 --timeout-method thread > $F/g2_tests.log 2>&1 || { tail -40 $F/g2_tests.log; exit 1; }
tail -2 $F/g2_tests.log
timeout -k 10 300 python bench.py --headline-only --no-cpu > $F/c2_g2.json 2> $F/c2_g2.err || exit $?
timeout -k 10 300 python bench.py --mode rowshard --steps 10 --warmup 5 > $F/rowshard_n1_g2.json 2> $F/rowshard_n1_g2.err || exit $?
rm -rf gpurun_out/pmc; bash scripts/pmc.sh > $F/pmc_g2.log 2>&1 || exit $?
python3 scripts/pmc_step.py gpurun_out/pmc 5 --json $F/pmc_c2_g2.json > /dev/null
python3 scripts/pmc_summary.py gpurun_out/pmc "eval_kernel<float, 16, 2, 0, true>" --json $F/pmc_c2_dispatch_g2.json > /dev/null
echo done
