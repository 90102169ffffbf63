#!/bin/bash
# Round-6 GPU loop on the product build: per-config call timing, then a GPU
# test subset (K: pytest -k expression).
#   OUT=r6g CFGS="libsvm dirty" K="dirty_rows" bash tools/gpu_r6b.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${OUT:-r6g}; mkdir -p $O
cd $R
for cfg in ${CFGS:-libsvm}; do
  timeout -k 10 120 python tools/time_variant.py $cfg 2>&1 | grep -v amdgpu.ids | tee -a $O/time.txt || exit 1
done
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?
  tail -3 $O/pytest.log
  [ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/pytest.log | head -30; exit $rc; }
fi
echo r6b done
