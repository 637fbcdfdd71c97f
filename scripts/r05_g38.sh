# round 5 GPU call 38: decision records prefetched during the wait (fresh-population pipeline A/B),
# the derived-view test with a batched view
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/g38
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py -x -q --timeout 300 --timeout-method thread -m gpu -k "derived or uniform" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ENVS="SRHIP_NO_DEC_PREFETCH=1;SRHIP_NO_DEC_PREFETCH=0" REPS=3 bash scripts/pipe_ab.sh | tee $O/pipe_ab.log
