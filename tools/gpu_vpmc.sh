#!/bin/bash
# VALU / SALU / LDS instructions per wave of ablation variants (one PMC pass each):
#   OUT=r6f VARS="full_abl0 ..." [CFG=libsvm] [KSUB=svm_fast_tile] bash tools/gpu_vpmc.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${OUT:-r6f}; mkdir -p $O
for v in ${VARS}; do
  lib=$R/dmlc-core_amd/lib/variants/$v.so; [ "$v" = default ] && lib=$R/dmlc-core_amd/lib/libdmlc_amd.so
  (cd /tmp && export TMPDIR=/tmp && DMLC_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM --kernel-trace --output-format csv -d $O/$v -o run -- python3 $R/tools/time_variant.py ${CFG:-libsvm} > $O/$v.log 2>&1) || { echo "pmc $v failed"; exit 1; }
  echo "== $v $(grep tile= $O/$v.log)"
  python3 $R/tools/pmc_read.py $O/$v ${KSUB:-svm_fast_tile} | grep -E "VALU|SALU|LDS|VMEM|WAVE_CYCLES"
done
