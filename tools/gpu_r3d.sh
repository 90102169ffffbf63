set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
for v in base; do DMLC_AMD_LIB=$GRAFT_REPO_ROOT/dmlc-core_amd/lib/variants/$v.so timeout -k 10 120 python tools/time_variant.py libsvm || exit 1; done
timeout -k 10 120 python tools/time_variant.py libsvm || exit 1
timeout -k 10 120 python tools/time_variant.py csv || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $O/abl/new1 -o run -- python3 $GRAFT_REPO_ROOT/tools/time_variant.py libsvm > $O/abl/new1.log 2>&1) || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest_r3d.log 2>&1; rc=$?; tail -3 $O/pytest_r3d.log; exit $rc
