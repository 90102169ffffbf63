#!/bin/bash
# GPU-box: time ablation variants (tools/build_variants.sh) with tools/time_variant.py.
# usage: VARIANTS="base nodec" [FMT=csv] bash tools/ablate.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in ${VARIANTS}; do
  DMLC_AMD_LIB=$R/dmlc-core_amd/lib/variants/$v.so timeout -k 10 120 python tools/time_variant.py ${FMT:-libsvm} || exit 1
done
