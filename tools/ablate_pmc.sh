#!/bin/bash
# GPU-box: SQ instruction counters per ablation variant (one --pmc pass each).
# usage: VARIANTS="base stop0 ..." bash tools/ablate_pmc.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abpmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS}; do
  DMLC_AMD_LIB=$R/dmlc-core_amd/lib/variants/$v.so timeout -s KILL 120 rocprofv3 --pmc ${COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES} --kernel-trace --output-format csv -d $O/$v${SFX} -o run -- python3 $R/tools/time_variant.py ${FMT:-libsvm} > $O/$v${SFX}.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  python3 - "$O/$v${SFX}" "$v${SFX}" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(list)
for row in csv.DictReader(open(f[0])):
    if "svm_fast_tile<2>" in row["Kernel_Name"] or "csv_fast_tile<2>" in row["Kernel_Name"]:
        acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
w = sum(acc["SQ_WAVES"]) / max(len(acc["SQ_WAVES"]), 1)
print(sys.argv[2], " ".join("%s=%.0f" % (k[3:], sum(v) / len(v) / w) for k, v in sorted(acc.items()) if k != "SQ_WAVES"), "waves=%.0f" % w)
PY
done
