#!/bin/bash
# Latency / issue-mix PMC passes of one variant (tools/time_variant.py), each
# pass its own rocprofv3 run:  V=base FMT=libsvm bash tools/pmc_lat.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/lat; mkdir -p $O
V=${V:-base}
LIB=$R/dmlc-core_amd/lib/variants/$V.so
[ -f $LIB ] || LIB=$R/dmlc-core_amd/lib/libdmlc_amd.so
i=0
for set in "SQ_WAVES SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" \
           "SQ_WAVES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS" \
           "SQ_WAVES SQ_INST_CYCLES_SALU SQ_LEVEL_WAVES SQ_BUSY_CU_CYCLES SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && DMLC_AMD_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/${V}_$i -o run -- python3 $R/tools/time_variant.py ${FMT:-libsvm} > $O/${V}_$i.log 2>&1) || { echo "pass $i failed"; exit 1; }
done
echo lat done
