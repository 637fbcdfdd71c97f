# round 5 GPU call 33: compact per-tree decisions + precise scratch ensured before the launch:
# precise tests, then the pipeline section with per-call host timing
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/g33
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_precise.py -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ENVS="SRHIP_X=0;SRHIP_HOST_TIMING=2" REPS=1 bash scripts/pipe_ab.sh || exit 1
cp gpurun_out/pipeab/2.1.err $O/host_timing.err
