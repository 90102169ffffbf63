"""Per-call GPU timeline of a rocprofv3 --kernel-trace run: each kernel's
duration and the gap before it (ns), for the last few dmlc_amd_parse calls.
usage: python tools/trace_gaps.py <kernel_trace.csv> [n_last_kernels]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
prev_end = None
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = s - prev_end if prev_end is not None else 0
    print("%8.1f us gap  %9.1f us  %s" % (gap / 1e3, (e - s) / 1e3, r["Kernel_Name"][:90]))
    prev_end = e
