# round 5 GPU call 28: C2 bench with per-population kernel times in the fresh-population pipeline
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/g28
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu > $O/bench_$rep.log 2>&1 || { tail -5 $O/bench_$rep.log; exit 1; }
  tail -1 $O/bench_$rep.log > $O/bench_$rep.json
  python3 -c "
import json; d=json.load(open('$O/bench_$rep.json')); p=d['extra']['population_pipeline']
print('kernel', round(d['roofline']['kernel_ms'],4), 'step', round(d['ms_per_step'],4), {k: (round(v,4) if isinstance(v,float) else v) for k,v in p.items() if k not in ('note',)})"
done
