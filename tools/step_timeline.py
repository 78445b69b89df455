#!/usr/bin/env python3
"""One bench step's kernel timeline from a rocprofv3 kernel trace:
tools/step_timeline.py <dir with run_kernel_trace.csv> [marker kernel]
Prints start offset, duration and the idle gap before every kernel of the
second-to-last step (steps delimited by the marker kernel, wc_hot_sample)."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
marker = sys.argv[2] if len(sys.argv) > 2 else "wc_hot_sample"
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = idx[-3], idx[-2]
t0 = int(rows[a]["Start_Timestamp"])
prev = None
busy = 0
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    if r is not rows[b]:
        busy += e - s
    print("%8.2f %8.2f gap=%6.2f %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, r["Kernel_Name"][:64]))
    prev = e
span = (int(rows[b]["Start_Timestamp"]) - t0) / 1e3
print("step span %.2f us, kernels busy %.2f us, idle %.2f us" % (span, busy / 1e3, span - busy / 1e3))
