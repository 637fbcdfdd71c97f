#!/bin/bash
# Round 4: native RCCL communicator tests (world 1), rowshard bench through srhip_eval_loss_sharded,
# then a same-box A/B of library builds (BUILDS) on the C2 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -v --timeout 120 --timeout-method thread > gpurun_out/comm_tests.log 2>&1
rc=$?; echo "comm tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/comm_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc  # a failing comm test (rc 1) stops the script too
timeout -k 10 300 python -u bench.py --mode rowshard --steps 10 --warmup 5 > gpurun_out/rowshard_n1.log 2>&1
rc=$?; echo "rowshard rc=$rc"; tail -1 gpurun_out/rowshard_n1.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
[ -n "${BUILDS:-}" ] && bash scripts/ab2.sh
