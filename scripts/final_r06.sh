#!/bin/bash
# Round-6 evidence on the committed build, one GPU session: GPU suite, smoke, C2 bench (CPU baseline),
# the headline kernel trace + per-step PMC passes, the row-shard line, C4 bench (all-core CPU baseline)
# + gradient PMC, C1 / C3 search lines, the multi-rank rehearsal, the native coalescer driver and the
# host-sanitizer driver's device phase.  Each step under its own time limit; stops at the first
# failure.  ONLY="c2 trace pmc" runs a subset; F=<dir> puts the outputs elsewhere.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${F:-gpurun_out/final6}
mkdir -p $F
export TMPDIR=/tmp
want() { [ -z "${ONLY:-}" ] || [[ " $ONLY " == *" $1 "* ]]; }
step() { echo "== $1"; }
if want tests; then
  step tests
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -30 $F/gpu_tests.log; exit 1; }
  tail -1 $F/gpu_tests.log
fi
if want smoke; then
  step smoke
  timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || exit $?
  tail -2 $F/smoke.log
fi
if want c2; then
  step c2
  timeout -k 10 400 python -u bench.py > $F/bench_c2.log 2>&1 || exit $?
  tail -1 $F/bench_c2.log > $F/bench_c2.json
fi
if want trace; then
  step trace
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $F/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 30 --no-cpu --headline-only > $F/prof.log 2>&1 || exit $?
  python3 scripts/trace_summary.py $F/prof/run_kernel_trace.csv > $F/trace_c2.txt; python3 scripts/step_timeline.py $F/prof/run_kernel_trace.csv 30 20 > $F/step_timeline_c2.txt
  python3 scripts/trace_timed_region.py $F/prof/run_kernel_trace.csv 20 30 > $F/trace_c2_timed_region.txt 2>&1 || true
  head -5 $F/trace_c2.txt
fi
if want pmc; then
  step pmc
  rm -rf gpurun_out/pmc; bash scripts/pmc.sh > $F/pmc.log 2>&1 || exit $?
  python3 scripts/pmc_step.py gpurun_out/pmc 8 --json $F/pmc_c2.json > /dev/null; python3 scripts/pmc_summary.py gpurun_out/pmc "eval_kernel<float, 16, 2, 0, true>" --json $F/pmc_c2_dispatch.json > /dev/null; cp -r gpurun_out/pmc $F/pmc_csv
fi
if want host; then
  step host
  bash scripts/host_timing.sh > $F/host_timing.log 2>&1 || exit $?
fi
if want rowshard; then
  step rowshard
  timeout -k 10 300 python -u bench.py --mode rowshard --steps 10 --warmup 5 > $F/rowshard_n1.log 2>&1 || exit $?
  tail -1 $F/rowshard_n1.log > $F/rowshard_n1.json
fi
if want c4; then
  step c4
  timeout -k 10 600 python -u bench.py --config c4 > $F/bench_c4.log 2>&1 || exit $?
  tail -1 $F/bench_c4.log > $F/bench_c4.json
fi
if want pmc_grad; then
  step pmc_grad
  rm -rf gpurun_out/pmcg; bash scripts/pmc_grad.sh > $F/pmc_grad.log 2>&1 || exit $?
  python3 scripts/pmc_step.py gpurun_out/pmcg 8 grad_kernel --json $F/pmc_grad_c4.json > /dev/null
fi
if want c1; then
  step c1
  timeout -k 10 400 python -u bench.py --config c1 > $F/bench_c1.log 2>&1 || exit $?
  tail -1 $F/bench_c1.log > $F/bench_c1.json
fi
if want c3; then
  step c3
  timeout -k 10 400 python -u bench.py --config c3 > $F/bench_c3.log 2>&1 || exit $?
  tail -1 $F/bench_c3.log > $F/bench_c3.json
fi
if want multi; then
  step multi
  bash scripts/multi_rehearsal.sh > $F/multi.log 2>&1 || exit $?
  cp gpurun_out/multi_*.json $F/
fi
if want coalescer; then
  step coalescer
  SECONDS_PER_RUN=3 timeout -k 10 200 python -u scripts/coalescer_native.py c3 16 64 > $F/coalescer_c3.jsonl 2>&1 || exit $?
  SECONDS_PER_RUN=3 timeout -k 10 200 python -u scripts/coalescer_native.py c1 1 16 64 > $F/coalescer_c1.jsonl 2>&1 || exit $?
fi
if want asan; then
  step asan
  LSAN_OPTIONS=suppressions=$PWD/tools/lsan_rocm.supp timeout -k 10 300 tools/build/host_stress_asan 8 20 > $F/host_stress_asan.log 2>&1 || { tail -30 $F/host_stress_asan.log; exit 1; }
  tail -1 $F/host_stress_asan.log
fi
if want probes; then
  step probes
  timeout -k 10 200 python -u scripts/compile_probe.py > $F/compile_probe.json 2> $F/compile_probe.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace -d $F/c4trace -o run --output-format csv -- python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu > $F/c4trace.log 2>&1 || exit $?
  python3 scripts/c4_trace.py $F/c4trace/run_kernel_trace.csv --json $F/c4_trace.json > /dev/null || exit $?
fi
echo done
