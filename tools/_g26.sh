set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g26; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --list-avail > $O/avail.txt 2>&1; echo "list rc=$?"
grep -o -E "SQC?_[A-Z0-9_]*(ICACHE|IFETCH|INST_LEVEL|WAIT_INST|LEVEL_INST|INSTS_BRANCH|INST_CYCLES)[A-Z0-9_]*" $O/avail.txt | sort -u > $O/names.txt; cat $O/names.txt
C=$(grep -E "^SQC_ICACHE_(HITS|MISSES|MISSES_DUPLICATE|REQ)$" $O/names.txt | sort -u | tr '\n' ' ')
echo "counters: $C"
[ -n "$C" ] || exit 0
timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/ic -o run -- python3 $R/tools/time_variant.py libsvm > $O/ic.log 2>&1; echo "pmc rc=$?"
python3 - $O/ic <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(list)
for row in csv.DictReader(open(f[0])):
    if "svm_fast_tile<2>" in row["Kernel_Name"]:
        acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, v in sorted(acc.items()): print(k, sum(v) / len(v))
PY
