#!/bin/bash
# VGPR count and occupancy per device function of the eval kernels (compile remarks, no GPU).
# usage: scripts/vgprs.sh [regex]   (default: the Float32 R=8 kernels and heavy bodies)
cd "$(dirname "$0")/../symbolicregression.jl_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize \
  -mllvm -structurizecfg-skip-uniform-regions=true -mllvm -disable-machine-licm ${EXTRA:-} \
  --cuda-device-only -c csrc/srhip_eval_${SLICE:-f32w}.hip -o /tmp/vgprs_eval.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n 's/.*remark: *//p' | awk -v pat="${1:-IfLi8E}" '
    /^Function Name:/ {name=$3; keep = (name ~ pat)}
    keep && /^VGPRs:/ {print name, "vgpr=" $2}
    keep && /^Occupancy/ {print name, "occ=" $3}'
