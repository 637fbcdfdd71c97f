# round 5 GPU call 19: list-overflow undecided trees through the device precise pass -- precise / parity
# suites, then the C2 bench's fresh-population pipelines
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_precise.py tests/test_gpu_parity.py tests/test_gpu_persistent.py tests/test_gpu_configs.py tests/test_gpu_batch_seams.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/g19_tests.log 2>&1 || { tail -30 $O/g19_tests.log; exit 1; }
tail -1 $O/g19_tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu > $O/c2_g19_$r.json 2> $O/c2_g19_$r.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/c2_g19_$r.json').read().strip().splitlines()[-1]); pp=d['extra']['population_pipeline']; print(d['ms_per_step'], pp['pipelined_phases_ms'], pp['sequential_ms_per_population'], pp['pipelined_ms_per_population'], pp['two_stream_ms_per_population'])"
done
