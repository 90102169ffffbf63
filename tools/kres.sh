#!/bin/bash
# Per-kernel resource usage (VGPRs, SGPRs, scratch, LDS) of a HIP source: tools/kres.sh csrc/libsvm.hip [-DFLAGS]
f=$1; shift
cd "$(dirname "$0")/../dmlc-core_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
  -I../include -Icsrc "$@" --cuda-device-only -S $f -o /tmp/kres.s 2>/dev/null
awk '/^\s+\.name:/{n=$2} /\.vgpr_count:/{v=$2} /\.sgpr_count:/{sg=$2} /\.private_segment_fixed_size:/{p=$2} /\.group_segment_fixed_size:/{l=$2} /\.vgpr_spill_count:/{print n, "vgpr", v, "sgpr", sg, "scratch", p, "lds", l, "vspill", $2}' /tmp/kres.s
