#!/bin/bash
# The N > 1 bench paths rehearsed on ONE GPU: two ranks sharing the device over gloo (RCCL cannot put
# two ranks on one GPU), C2 islands (per-step migration all-gather) and rowshard (per-step partials
# all-reduce); plus rowshard at N = 1.  Outputs gpurun_out/multi_*.json; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --mode rowshard --steps ${STEPS:-5} --warmup 2 > gpurun_out/multi_rowshard_n1.log 2>&1 || exit $?
tail -1 gpurun_out/multi_rowshard_n1.log | tee gpurun_out/multi_rowshard_n1.json | cut -c1-600
for mode in islands rowshard; do
  SRHIP_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29633 bench.py --gpus 2 --mode $mode --steps ${STEPS:-5} --warmup 2 --no-cpu \
    --headline-only > gpurun_out/multi_${mode}_n2.log 2>&1 || exit $?
  grep '^{' gpurun_out/multi_${mode}_n2.log | tail -1 | tee gpurun_out/multi_${mode}_n2.json | cut -c1-600
done
