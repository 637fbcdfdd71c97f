# round 5 GPU call 18: the C2 bench's single-context pipeline, phase by phase
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu > $O/c2_g18_$r.json 2> $O/c2_g18_$r.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/c2_g18_$r.json').read().strip().splitlines()[-1]); pp=d['extra']['population_pipeline']; print(pp['pipelined_phases_ms'], pp['sequential_ms_per_population'], pp['pipelined_ms_per_population'], pp['two_stream_ms_per_population'])"
done
