# round 5 GPU call 13: comm self-check comparisons at world 1, and the C2 bench's fresh-population
# pipelines (one stream / two streams)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/g13_comm.log 2>&1 || { tail -30 $O/g13_comm.log; exit 1; }
tail -1 $O/g13_comm.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu > $O/c2_g13_$r.json 2> $O/c2_g13_$r.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/c2_g13_$r.json').read().strip().splitlines()[-1]); pp=d['extra']['population_pipeline']; print(d['ms_per_step'], d['roofline']['kernel_ms'], {k: pp[k] for k in pp if k.endswith('ms') or k.endswith('population')})"
done
