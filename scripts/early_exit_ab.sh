#!/bin/bash
# GPU suite, then the C2 bench with and without the early exit of failed trees.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  SRHIP_NO_EARLY_EXIT=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_ee$v.json 2> gpurun_out/bench_ee$v.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_ee$v.json'));r=d['roofline'];print('NO_EARLY_EXIT=$v', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'])"
done
