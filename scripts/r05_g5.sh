# round 5 GPU call 5: the fresh-population pipeline -- where its time goes beside the kernel (pool
# workers' priority, compile threads)
set -u
cd $GRAFT_REPO_ROOT
F=gpurun_out/r05
mkdir -p $F
for e in "" "SRHIP_POOL_NICE=10" "SRHIP_COMPILE_THREADS=8" "SRHIP_COMPILE_THREADS=4" "SRHIP_POOL_NICE=10 SRHIP_COMPILE_THREADS=8"; do
  env $e timeout -k 10 200 python scripts/pipeline_probe.py >> $F/pipeline_probe_g5.jsonl 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --no-cpu > $F/c2_g5.json 2> $F/c2_g5.err || exit $?
echo done
