#!/usr/bin/env python3
"""H2D copy vs kernel overlap from a rocprofv3 --kernel-trace --memory-copy-trace CSV directory.

usage: tools/copy_overlap.py gpurun_out/prof_file [TEXT_BYTES]
Prints copy count / bytes / busy time / achieved GB/s, kernel busy time, and how much of the
copy time ran while a wc_map / wc_reduce kernel was executing (union of intervals)."""
import csv
import glob
import os
import sys


def load(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def overlap(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        lo, hi = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        tot += max(0, hi - lo)
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


d = sys.argv[1]
kt = load(d, "*kernel_trace.csv")
mc = load(d, "*memory_copy_trace.csv")
# this rocprofv3 build has no Size column: text pieces are the H2D copies longer than 100 us
# (the per-pass counter copies take a few us); bytes = --bytes / copies when given
h2d = [r for r in mc if "HOST_TO_DEVICE" in r.get("Direction", "")
       and int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 100_000]
ker = [r for r in kt if r["Kernel_Name"].startswith(("wc::dev::wc_map", "wc::dev::wc_reduce", "void wc::dev::wc_map"))]
ci = union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in h2d])
ki = union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ker])
cb = sum(b - a for a, b in ci)
kb = sum(b - a for a, b in ki)
nbytes = int(sys.argv[2]) if len(sys.argv) > 2 else 0
span = (max(b for _, b in ci + ki) - min(a for a, _ in ci + ki)) if ci and ki else 0
print(f"H2D text copies: {len(h2d)}, {nbytes / 2**30:.2f} GiB, busy {cb / 1e6:.1f} ms "
      f"({nbytes / max(cb, 1):.2f} GB/s while copying)")
print(f"map/reduce kernels: {len(ker)} dispatches, busy {kb / 1e6:.1f} ms")
print(f"copy time overlapped with kernels: {overlap(ci, ki) / 1e6:.1f} ms; first copy -> last kernel span {span / 1e6:.1f} ms")
