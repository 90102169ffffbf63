set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/${OUT:-r6b}
for v in ${VARS:-lean_abl1 lean_abl2 lean_w5 full_abl2}; do
  DMLC_AMD_LIB=dmlc-core_amd/lib/variants/$v.so timeout -k 10 120 python tools/time_variant.py libsvm 2>&1 | grep tile= | tee -a gpurun_out/${OUT:-r6b}/time.txt || exit 1
done
DMLC_AMD_LEAN=1 timeout -k 10 120 python tools/time_variant.py libsvm 2>&1 | grep tile= | tee -a gpurun_out/${OUT:-r6b}/time.txt
