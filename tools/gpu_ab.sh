#!/bin/bash
# A/B timing of variant libraries (tools/build_variants.sh) with
# tools/time_variant.py, plus one PMC instruction pass per variant.
#   VARIANTS="base new" [FMT=libsvm] [PMC=1] bash tools/gpu_ab.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab; mkdir -p $O
cd $R
for pass in 1 2; do
  for v in $VARIANTS; do
    DMLC_AMD_LIB=$R/dmlc-core_amd/lib/variants/$v.so timeout -k 10 120 python tools/time_variant.py ${FMT:-libsvm} || exit 1
  done
done
[ -n "$PMC" ] || exit 0
for v in $VARIANTS; do
  (cd /tmp && export TMPDIR=/tmp && DMLC_AMD_LIB=$R/dmlc-core_amd/lib/variants/$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $O/$v -o run -- python3 $R/tools/time_variant.py ${FMT:-libsvm} > $O/$v.log 2>&1) || { echo "pmc $v failed"; exit 1; }
done
echo ab done
