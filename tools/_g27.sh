set -o pipefail
VARIANTS="base stop0 stop1 stop2 stop3 nodec nostore" COUNTERS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES" bash tools/ablate_pmc.sh || exit 1
for v in base stop0 stop1 stop2 stop3 nodec nostore; do DMLC_AMD_LIB=$GRAFT_REPO_ROOT/dmlc-core_amd/lib/variants/$v.so timeout -k 10 120 python tools/time_variant.py libsvm || exit 1; done
