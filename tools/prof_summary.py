#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel stats / PMC counters) as markdown.

usage: tools/prof_summary.py gpurun_out/prof7 [--title T] > profiles/xyz.md
"""
import argparse
import collections
import csv
import glob
import os


def kernel_stats(d):
    f = glob.glob(os.path.join(d, "*kernel_stats.csv"))
    if not f:
        return ""
    rows = list(csv.DictReader(open(f[0])))
    out = ["| kernel | calls | avg (us) | total (ms) | % |", "|---|---:|---:|---:|---:|"]
    for r in rows:
        name = r["Name"].split("(")[0]
        out.append(f"| `{name}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                   f"{float(r['TotalDurationNs'])/1e6:.3f} | {float(r['Percentage']):.1f} |")
    return "\n".join(out)


def counters(d):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not f:
        return ""
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    out = []
    for k, v in agg.items():
        n = len(disp[k])
        out.append(f"**`{k}`** (per dispatch, {n} dispatches)\n")
        out.append("| counter | value |\n|---|---:|")
        out += [f"| {c} | {val / n:.4g} |" for c, val in sorted(v.items())]
        out.append("")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--title", default="rocprofv3 summary")
    a = ap.parse_args()
    print(f"# {a.title}\n")
    for d in a.dirs:
        print(f"## {d}\n")
        ks, cs = kernel_stats(d), counters(d)
        if ks:
            print(ks + "\n")
        if cs:
            print(cs + "\n")


if __name__ == "__main__":
    main()
