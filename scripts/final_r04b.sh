#!/bin/bash
# Round-4 closing evidence after the block-counter change (committed build): smoke, C2 bench (CPU
# baseline), the headline kernel trace + per-step and per-dispatch PMC, host timing, the native
# coalescer, C3 / C1 search lines.  Each step under its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final2
export TMPDIR=/tmp
F=gpurun_out/final2
step() { echo "== $1"; }
step smoke
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || exit $?
tail -1 $F/smoke.log
step c2
timeout -k 10 400 python -u bench.py > $F/bench_c2.log 2>&1 || exit $?
tail -1 $F/bench_c2.log > $F/bench_c2.json
step trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $F/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 30 --no-cpu --headline-only > $F/prof.log 2>&1 || exit $?
python3 scripts/trace_summary.py $F/prof/run_kernel_trace.csv > $F/trace_c2.txt; python3 scripts/step_timeline.py $F/prof/run_kernel_trace.csv > $F/step_timeline_c2.txt; head -5 $F/trace_c2.txt
step pmc
rm -rf gpurun_out/pmc; bash scripts/pmc.sh > $F/pmc.log 2>&1 || exit $?
python3 scripts/pmc_step.py gpurun_out/pmc 5 --json $F/pmc_c2.json > /dev/null; python3 scripts/pmc_summary.py gpurun_out/pmc "eval_kernel<float, 16, 2, 0, true>" --json $F/pmc_c2_dispatch.json > /dev/null; cp -r gpurun_out/pmc $F/pmc_csv
step host
bash scripts/host_timing.sh > $F/host_timing.log 2>&1 || exit $?
step coalescer
SECONDS_PER_RUN=3 timeout -k 10 200 python -u scripts/coalescer_native.py c3 16 64 > $F/coalescer_c3.jsonl 2>&1 || exit $?
SECONDS_PER_RUN=3 timeout -k 10 200 python -u scripts/coalescer_native.py c1 1 16 64 > $F/coalescer_c1.jsonl 2>&1 || exit $?
step c3
timeout -k 10 400 python -u bench.py --config c3 > $F/bench_c3.log 2>&1 || exit $?
tail -1 $F/bench_c3.log > $F/bench_c3.json
step c1
timeout -k 10 400 python -u bench.py --config c1 > $F/bench_c1.log 2>&1 || exit $?
tail -1 $F/bench_c1.log > $F/bench_c1.json
echo done
