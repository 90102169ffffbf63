set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/abl; mkdir -p $O
for v in base stop0 stop1 stop2 stop3 nodec nostore; do
  DMLC_AMD_LIB=$GRAFT_REPO_ROOT/dmlc-core_amd/lib/variants/$v.so timeout -k 10 120 python tools/time_variant.py libsvm || exit 1
done
for v in base stop0 stop1 stop2 stop3 nodec nostore; do
  (cd /tmp && export TMPDIR=/tmp && DMLC_AMD_LIB=$GRAFT_REPO_ROOT/dmlc-core_amd/lib/variants/$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $O/$v -o run -- python3 $GRAFT_REPO_ROOT/tools/time_variant.py libsvm > $O/$v.log 2>&1) || { echo "pmc $v failed"; exit 1; }
done
echo abl done
