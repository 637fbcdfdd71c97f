# A/B of the launch's tail-shaped tree groups (srhip_host.cpp shape_groups tuning hooks)
set -u
run() { tag=$1; shift; env "$@" timeout -k 10 120 python3 bench.py --no-cpu --steps 20 > gpurun_out/sw_$tag.log 2>&1 || exit 1; }
run notail SRHIP_NO_TAIL=1
run d32 SRHIP_TAIL_DIV=32
run d64 SRHIP_TAIL_DIV=64
run d48 SRHIP_TAIL_DIV=48
run d32m32 SRHIP_TAIL_DIV=32 SRHIP_TAIL_MIN=32
run d16m64 SRHIP_TAIL_DIV=16 SRHIP_TAIL_MIN=64
run d32g1 SRHIP_TAIL_DIV=32 SRHIP_BULK_GROUPS=1
run d64g1 SRHIP_TAIL_DIV=64 SRHIP_BULK_GROUPS=1
run d24 SRHIP_TAIL_DIV=24
run notail2 SRHIP_NO_TAIL=1
run d32b SRHIP_TAIL_DIV=32
