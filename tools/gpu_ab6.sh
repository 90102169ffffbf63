#!/bin/bash
# A/B timing of variant libraries (lib/variants/<v>.so) on the libsvm configs,
# each timed twice, interleaved.  usage: VARS="a b" CFGS="libsvm cmt" bash tools/gpu_ab6.sh [tag]
set -o pipefail
TAG=${1:-r6_ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
for rep in 1 2; do for cfg in ${CFGS:-libsvm}; do for v in ${VARS}; do
  DMLC_AMD_LIB=dmlc-core_amd/lib/variants/$v.so timeout -k 10 120 python tools/time_variant.py $cfg 2>&1 | grep tile= | sed "s/^/$cfg /" | tee -a $O/time.txt || exit 1
done; done; done
