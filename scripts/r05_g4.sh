# round 5 GPU call 4: the whole GPU suite after the program pool / deferred teardown / planned order;
# C2 with its population pipeline; the pipeline probe; per-operator costs with Julia's trig
set -u
cd $GRAFT_REPO_ROOT
F=gpurun_out/r05
mkdir -p $F
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $F/g4_tests.log 2>&1 || { tail -40 $F/g4_tests.log; exit 1; }
tail -1 $F/g4_tests.log
timeout -k 10 300 python bench.py --no-cpu > $F/c2_g4.json 2> $F/c2_g4.err || exit $?
timeout -k 10 200 python scripts/pipeline_probe.py > $F/pipeline_probe_g4.json 2>&1 || exit $?
bash scripts/op_costs.sh > $F/op_costs_g4.log 2>&1 || exit $?
cp gpurun_out/opc/op_costs.json $F/op_costs_g4.json
echo done
