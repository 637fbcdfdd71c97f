# round 5 GPU call 1: Julia Float32 trig by default -- the GPU suite, the headline, the --gpus 2 launcher
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05/gpu_tests_g1.log 2>&1 && \
timeout -k 10 300 python bench.py --headline-only --no-cpu > gpurun_out/r05/c2_jtrig_g1.json 2> gpurun_out/r05/c2_jtrig_g1.err && \
SRHIP_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 10 --headline-only --no-cpu > gpurun_out/r05/islands_gloo_n2.json 2> gpurun_out/r05/islands_gloo_n2.err && \
timeout -k 10 200 python scripts/pipeline_probe.py > gpurun_out/r05/pipeline_probe_g1.json 2>&1
