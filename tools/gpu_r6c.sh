#!/bin/bash
# Round-6 state check on the product build: lean vs full call timing per
# libsvm config, the default bench line, then the whole GPU suite.
#   OUT=r6c [CFGS="libsvm dirty"] [SUITE=1] bash tools/gpu_r6c.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${OUT:-r6c}; mkdir -p $O
cd $R
for cfg in ${CFGS:-libsvm qid cmt hdrs dirty}; do
  for lean in 1 0; do
    DMLC_AMD_LEAN=$lean timeout -k 10 120 python tools/time_variant.py $cfg 2>&1 | grep -v amdgpu.ids | sed "s/^/lean=$lean $cfg /" | tee -a $O/time.txt || exit 1
  done
done
for cfg in ${CCFGS:-csv csv_dirty}; do
  timeout -k 10 120 python tools/time_variant.py $cfg 2>&1 | grep -v amdgpu.ids | sed "s/^/$cfg /" | tee -a $O/time.txt || exit 1
done
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
if [ -n "$SUITE" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?
  tail -3 $O/pytest.log
  [ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/pytest.log | head -30; exit $rc; }
fi
echo r6c done
