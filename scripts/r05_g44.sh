# round 5 GPU call 44: optimiser launches without timing events: optimiser tests, C4 bench x3
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/g44
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_derivatives.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  timeout -k 10 600 python -u bench.py --config c4 --no-cpu > $O/c4_$rep.log 2>&1 || { tail -5 $O/c4_$rep.log; exit 1; }
  tail -1 $O/c4_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['improved_trees'])"
done
