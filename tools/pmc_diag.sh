#!/bin/bash
# Diagnostic PMC passes (instruction cache, issue / wait breakdown, LDS) over
# tools/time_variant.py for the default library or DMLC_AMD_LIB; one counter
# group per rocprofv3 run.  usage: TAG=x [FMT=libsvm] bash tools/pmc_diag.sh
set -o pipefail
TAG=${TAG:-diag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmcd_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$name -o run -- \
    python3 $R/tools/time_variant.py ${FMT:-libsvm} > $O/$name.log 2>&1 || { echo "pass $name failed"; tail -3 $O/$name.log; return 1; }
}
run ic SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH \
 && run w1 SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES SQ_LDS_UNALIGNED_STALL \
 && run w2 SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_BUSY_CYCLES \
 && run w3 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_IFETCH_LEVEL SQ_ACTIVE_INST_ANY \
 && echo diag done
