"""Counter bytes / true bytes per access width from tools/pmc_calib.sh's
runs: python tools/pmc_calib_read.py gpurun_out/pmc_calib"""
import collections
import csv
import glob
import json
import sys

KIB = (1 << 30) >> 10  # pmc_calib.hip kBytes in KiB
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    per = collections.defaultdict(float)
    for f in glob.glob("%s/%s/**/run_counter_collection.csv" % (sys.argv[1], c), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == c:
                per[r["Kernel_Name"]] += float(r["Counter_Value"])
    for k, v in per.items():
        name = k.split("(")[0].replace("void ", "")
        if (c == "FETCH_SIZE") == name.startswith("read_w"):
            out["%s %s" % (c, name)] = round(v / KIB, 4)
print(json.dumps({"case": "pmc_calib", "counter_bytes_over_true_bytes": out}))
