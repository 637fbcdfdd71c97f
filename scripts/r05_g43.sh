# round 5 GPU call 43: reduce kernel with overlapped record loads: GPU suite, then the C2 kernel trace
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/g43
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 30 --no-cpu --headline-only > $O/prof.log 2>&1 || exit $?
python3 scripts/trace_summary.py $O/prof/run_kernel_trace.csv > $O/trace_c2.txt; head -6 $O/trace_c2.txt
