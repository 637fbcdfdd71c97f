# round 5 GPU call 42: C1 / C3 searches with worker processes (:multiprocessing, one context each)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/g42
mkdir -p $O
export TMPDIR=/tmp
for p in 8 16; do
  timeout -k 10 300 python -u bench.py --config c1 --parallelism multiprocessing --procs $p --no-cpu > $O/c1_mp$p.log 2>&1 || { tail -20 $O/c1_mp$p.log; exit 1; }
  tail -1 $O/c1_mp$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1 procs $p', d['value'], d.get('ms_per_step'))"
done
timeout -k 10 400 python -u bench.py --config c3 --parallelism multiprocessing --procs 15 --no-cpu > $O/c3_mp15.log 2>&1 || { tail -20 $O/c3_mp15.log; exit 1; }
tail -1 $O/c3_mp15.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 procs 15', d['value'], d.get('ms_per_step'))"
