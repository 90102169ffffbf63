"""Summarise a rocprofv3 kernel-trace --stats run and PMC passes into profiles/.

usage: python tools/summarize_prof.py <gpurun_out dir with prof_<tag>/ and pmc_<tag>/> <tag>

Writes profiles/<tag>_kernel_stats.csv (the rocprofv3 --stats summary, copied)
and profiles/<tag>_summary.json: per kernel the average duration, and for the
dominant kernel the HBM traffic per launch from FETCH_SIZE / WRITE_SIZE,
corrected as MI355X_MICROARCH.md prescribes for gfx950 (FETCH_SIZE counts half
the bytes of 16-byte-per-lane streaming reads, so it is doubled; WRITE_SIZE is
exact for 16-byte stores; both are in KiB).
"""
import collections
import csv
import json
import os
import shutil
import sys


def kernel_stats(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                          "pct": float(r["Percentage"])}
    return out


def pmc(path, kernel_substr):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if kernel_substr not in r["Kernel_Name"]:
            continue
        per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {c: sum(v.values()) / len(v) for c, v in per.items() if v}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = os.path.join(root, "profiles")
    os.makedirs(dst, exist_ok=True)
    summary = {"tag": tag}
    ks = os.path.join(src, "prof_%s" % tag, "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(dst, "%s_kernel_stats.csv" % tag))
        summary["kernels"] = kernel_stats(ks)
    dom = sys.argv[3] if len(sys.argv) > 3 else "svm_fast_tile<2>"
    counters = {}
    for sub in ("fetch", "write", "sq", "sq2"):
        p = os.path.join(src, "pmc_%s" % tag, sub, "run_counter_collection.csv")
        if os.path.exists(p):
            counters.update(pmc(p, dom))
    if counters:
        summary["dominant_kernel"] = dom
        summary["pmc_per_launch"] = counters
        if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
            fetch = counters["FETCH_SIZE"] * 1024 * 2  # KiB, x2: gfx950 half-count of wide reads
            write = counters["WRITE_SIZE"] * 1024
            summary["hbm_bytes_per_launch"] = {"read": fetch, "write": write, "total": fetch + write}
    json.dump(summary, open(os.path.join(dst, "%s_summary.json" % tag), "w"), indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1, sort_keys=True)[:3000])


if __name__ == "__main__":
    main()
