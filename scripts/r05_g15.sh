# round 5 GPU call 15: fresh-population pipelines -- evaluation streams (2 / 3) and compile threads (16 / 8)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/streams
mkdir -p $O
for rep in 1 2; do
  for e in "SRHIP_BENCH_STREAMS=2" "SRHIP_BENCH_STREAMS=3" "SRHIP_BENCH_STREAMS=2 SRHIP_COMPILE_THREADS=8" "SRHIP_BENCH_STREAMS=3 SRHIP_COMPILE_THREADS=8"; do
    tag=$(echo "$e" | tr ' =' '__')
    env $e timeout -k 10 300 python -u bench.py --no-cpu > $O/$tag.$rep.json 2> $O/$tag.$rep.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/$tag.$rep.json').read().strip().splitlines()[-1]); pp=d['extra']['population_pipeline']; print('$e', '%.3f' % d['roofline']['kernel_ms'], 'seq %.3f pipe %.3f streams %.3f fill %.3f' % (pp['sequential_ms_per_population'], pp['pipelined_ms_per_population'], pp['two_stream_ms_per_population'], pp['pipeline_fill_ms']))"
  done
done
