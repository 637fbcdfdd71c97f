#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/search
export TMPDIR=/tmp
for w in 300 0 50; do
  SRHIP_COALESCE_WAIT_US=$w timeout -k 10 120 python -u bench.py --config c1 --no-cpu > gpurun_out/search/c1_w$w.json 2> gpurun_out/search/c1_w$w.err || exit $?
  tail -c 600 gpurun_out/search/c1_w$w.json
done
for w in 300 0; do
  SRHIP_COALESCE_WAIT_US=$w timeout -k 10 200 python -u bench.py --config c3 --no-cpu > gpurun_out/search/c3_w$w.json 2> gpurun_out/search/c3_w$w.err || exit $?
  tail -c 600 gpurun_out/search/c3_w$w.json
done
