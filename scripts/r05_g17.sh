# round 5 GPU call 17: compile probe (main thread / worker thread / beside evaluations; the bench's
# single-context pipeline phase by phase)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python -u scripts/compile_probe.py > $O/compile_probe_$r.json 2> $O/compile_probe.err || { tail -20 $O/compile_probe.err; exit 1; }
  cat $O/compile_probe_$r.json
done
