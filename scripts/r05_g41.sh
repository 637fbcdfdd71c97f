# round 5 GPU call 41: SQC instruction / scalar data cache counters for the C2 headline kernel
# (one counter group per rocprofv3 pass, each pass under a hard timeout)
set -u
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc
PMC_LIST="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE
SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES
SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" bash scripts/pmc.sh || exit 1
mkdir -p gpurun_out/r05/g41 && cp -r gpurun_out/pmc gpurun_out/r05/g41/
python3 scripts/pmc_step.py gpurun_out/pmc 5 --json gpurun_out/r05/g41/pmc_sqc.json > /dev/null || true
python3 scripts/pmc_summary.py gpurun_out/pmc "eval_kernel<float, 16, 2, 0, true>" --json gpurun_out/r05/g41/pmc_sqc_dispatch.json > /dev/null || true
echo done
