# round 5 GPU call 46: the committed tree -- GPU suite, smoke, the default bench line
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/g46
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['cpu_baseline']['value'], d['extra']['population_pipeline']['pipelined_ms_per_population'])"
