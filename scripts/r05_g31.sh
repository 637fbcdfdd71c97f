# round 5 GPU call 31: precise list at full capacity with strided launch groups: GPU suite, then the
# C2 bench's fresh-population pipeline (twice) with per-call host timing on the second run
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/g31
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
ENVS="SRHIP_X=0;SRHIP_HOST_TIMING=2" REPS=1 bash scripts/pipe_ab.sh || exit 1
cp gpurun_out/pipeab/2.1.err $O/host_timing.err
