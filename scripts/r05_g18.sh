# round 5 GPU call 18: the C2 bench's single-context pipeline, phase by phase
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 300 python -u bench.py --no-cpu > $O/c2_g18.json 2> $O/c2_g18.err || exit $?
python3 -c "import json; d=json.loads(open('$O/c2_g18.json').read().strip().splitlines()[-1]); pp=d['extra']['population_pipeline']; print(json.dumps(pp))"
