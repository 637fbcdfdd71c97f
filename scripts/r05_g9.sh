# round 5 GPU call 9: C4 per-launch log of the caller's group (SRHIP_OPTIM_TIMING=3) and every evaluation of
# the slowest tree (SRHIP_OPTIM_TRACE=321)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/c4l
mkdir -p $O
SRHIP_OPTIM_TIMING=3 SRHIP_OPTIM_TRACE=321 timeout -k 10 300 python3 -u bench.py --config c4 --steps 1 --warmup 1 --no-cpu > $O/run.json 2> $O/run.err || exit $?
grep -c "srhip launch" $O/run.err
grep "srhip optim:" $O/run.err | tail -3
