# round 5 GPU call 16: GPU suite after the compiler changes (lazy cache entries, derived-program copy),
# then the C2 bench's fresh-population pipelines twice
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/g16_tests.log 2>&1 || { tail -30 $O/g16_tests.log; exit 1; }
tail -1 $O/g16_tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu > $O/c2_g16_$r.json 2> $O/c2_g16_$r.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/c2_g16_$r.json').read().strip().splitlines()[-1]); pp=d['extra']['population_pipeline']; print('%.3f %.3f' % (d['ms_per_step'], d['roofline']['kernel_ms']), {k: round(pp[k], 3) for k in pp if k.endswith('ms') or k.endswith('population')})"
done
