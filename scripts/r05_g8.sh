# round 5 GPU call 8: C4 where-does-the-time-go -- launch histogram (SRHIP_OPTIM_TIMING=2) and a kernel trace of
# one optimize_constants call at the default split (3 groups) and at split 1
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05/c4t
mkdir -p $O
SRHIP_OPTIM_TIMING=2 timeout -k 10 300 python3 -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu > $O/timing.json 2> $O/timing.err || exit $?
grep "srhip optim" $O/timing.err | tail -8
for g in 3 1; do
  SRHIP_OPTIM_SPLIT=$g timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace$g -o run --output-format csv -- \
    python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu > $O/trace$g.log 2>&1 || exit $?
  python3 scripts/c4_trace.py $O/trace$g/run_kernel_trace.csv --json $O/c4_trace_split$g.json > /dev/null || exit $?
  python3 -c "import json; d=json.load(open('$O/c4_trace_split$g.json')); print($g, d['span_ms'], d['busy_ms'], d['kernels'], d['launches_per_queue'])"
done
