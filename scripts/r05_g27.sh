# round 5 GPU call 27: the build after removing the gradient-record folding: GPU suite, C4 bench
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/g27
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python -u bench.py --config c4 --no-cpu > $O/bench_c4.log 2>&1 || { tail -5 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value'], d.get('ms_per_step'), d['roofline']['frac'])"
