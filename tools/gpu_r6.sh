#!/bin/bash
# Round-6 GPU loop: lean vs full single-pass timing on the libsvm configs,
# one PMC instruction pass per mode, then the GPU parity suite.
#   OUT=r6a [CFGS="libsvm qid"] [SUITE=1] [PMC=1] bash tools/gpu_r6.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${OUT:-r6}; mkdir -p $O
cd $R
for cfg in ${CFGS:-libsvm qid cmt hdrs}; do
  for lean in 1 0; do
    DMLC_AMD_LEAN=$lean timeout -k 10 120 python tools/time_variant.py $cfg 2>&1 | tee -a $O/time.txt || exit 1
  done
done
if [ -n "$PMC" ]; then
  for lean in 1 0; do
    (cd /tmp && export TMPDIR=/tmp && DMLC_AMD_LEAN=$lean timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $O/pmc_lean$lean -o run -- python3 $R/tools/time_variant.py libsvm > $O/pmc_lean$lean.log 2>&1) || { echo "pmc failed"; exit 1; }
  done
fi
if [ -n "$SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?
  tail -3 $O/pytest.log
  [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit $rc; }
fi
echo r6 done
