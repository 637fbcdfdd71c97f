# A/B of the launch's tail-shaped tree groups (srhip_host.cpp shape_groups tuning hooks)
set -u
run() { tag=$1; shift; env "$@" timeout -k 10 120 python3 bench.py --no-cpu --steps 20 > gpurun_out/sw_$tag.log 2>&1 || exit 1; }
run d32 SRHIP_TAIL_DIV=32
run g1 SRHIP_BULK_GROUPS=1
run g4 SRHIP_BULK_GROUPS=4
run d32b SRHIP_TAIL_DIV=32
