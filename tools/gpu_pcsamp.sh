#!/bin/bash
# PC sampling of the single-pass kernel (rocprofv3 stochastic sampling): which
# instructions of svm_fast_tile<2> the waves sit on, and why.
#   [FMT=libsvm] [LIBV=variant] bash tools/gpu_pcsamp.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pcs${LIBV:+_$LIBV}; mkdir -p $O
extra=()
[ -n "$LIBV" ] && export DMLC_AMD_LIB=$R/dmlc-core_amd/lib/variants/$LIBV.so
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${PCS_TIMEOUT:-240} rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${PCS_METHOD:-stochastic} \
  --pc-sampling-unit ${PCS_UNIT:-cycles} --pc-sampling-interval ${PCS_INTERVAL:-1048576} \
  --output-format csv -d $O -o run -- python3 $R/tools/time_variant.py ${FMT:-libsvm} > $O/log.txt 2>&1
rc=$?
tail -5 $O/log.txt
find $O -name "*.csv" | head
exit $rc
