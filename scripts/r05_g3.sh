# round 5 GPU call 3: program-buffer pool (pipeline probe), cos tier C on Cody-Waite alone (C2), the
# trig parity tests, C4 unchanged
set -u
cd $GRAFT_REPO_ROOT
F=gpurun_out/r05
mkdir -p $F
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_math.py tests/test_gpu_configs.py tests/test_gpu_persistent.py -x -q --timeout 240 --timeout-method thread > $F/g3_tests.log 2>&1 || { tail -40 $F/g3_tests.log; exit 1; }
tail -1 $F/g3_tests.log
timeout -k 10 300 python bench.py --no-cpu > $F/c2_g3.json 2> $F/c2_g3.err || exit $?
timeout -k 10 200 python scripts/pipeline_probe.py > $F/pipeline_probe_g3.json 2>&1 || exit $?
timeout -k 10 400 python bench.py --config c4 --no-cpu --steps 5 --warmup 2 > $F/c4_g3.json 2> $F/c4_g3.err || exit $?
echo done
