"""Average PMC counters per dispatch of one kernel from tools/pmc_diag.sh output.
usage: python tools/pmc_read.py gpurun_out/pmcd_<tag> [kernel substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 else "svm_fast_tile<2>"
acc = {}
for f in sorted(glob.glob(d + "/**/*counter_collection.csv", recursive=True)):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if ksub in r["Kernel_Name"]:
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, v in per.items():
        acc[c] = sum(v.values()) / len(v)
w = acc.get("SQ_WAVES", 0)
for k in sorted(acc):
    extra = " (per wave %.1f)" % (acc[k] / w) if w and k != "SQ_WAVES" else ""
    print("%-30s %16.1f%s" % (k, acc[k], extra))
