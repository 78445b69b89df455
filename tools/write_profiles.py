#!/usr/bin/env python3
"""Write profiles/<tag>_{kernels,sweep}.md from an evidence bundle (tools/evidence.sh output in gpurun_out/)."""
import json
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
title = sys.argv[2] if len(sys.argv) > 2 else tag
rows = [json.loads(l) for l in open("gpurun_out/sweep.jsonl")]
labels = ["1gb, Zipf(1.0) 100k vocab (headline)", "1gb, vocab 500", "1gb, vocab 10k", "1gb, vocab 1M",
          "64gb config (64 GiB HBM-resident, 2 GiB chunks)", "host-staged (16 GiB replayed from a 4 GiB pinned pool)"]
out = [f"# {title}: config sweep on one MI355X (bench.py, gpurun_out/sweep.jsonl)", "",
       "| config | GB/s | ms/step | words/s | distinct | records after combiner |", "|---|---:|---:|---:|---:|---:|"]
for lab, d in zip(labels, rows):
    st = d["stages"]
    out.append(f"| {lab} | {d['value']:.1f} | {d['ms_per_step']:.2f} | {d['words_per_s']/1e9:.1f} G | "
               f"{d['distinct_words']} | {st['records']/1e6:.1f} M |")
out += ["", "Host-staged is bound by PCIe Gen5 x16 (63 GB/s spec)."]
open(f"profiles/{tag}_sweep.md", "w").write("\n".join(out) + "\n")
prof = open("gpurun_out/evidence_prof.txt").read()
phase = open("gpurun_out/evidence_phase.txt").read().strip().splitlines()
txt = [f"# {title}: kernel times and map phase clock (1 GiB Zipf-100k, bench.py --steps 5 --warmup 1)", "",
       "`rocprofv3 --kernel-trace --stats` (6 dispatches = 1 warmup + 5 steps; `wc_synth_text` is the one-time",
       "device text generation outside the timed region):", "", prof.split("## gpurun_out/prof_r1")[1].strip(), "",
       "## Map phase clock (`WC_MAP_STAMPS=1`: s_memtime laps per wave, accumulated in LDS)", "",
       "Shares of wave lifetime (diagnostic build).  `retry` = waiting at the flush barrier for the other waves",
       "to finish their current step (+ retries), `barrier` / `fl-write` = the flush itself.", "", "```",
       "zipf-100k: " + phase[0].split("] ")[1], "vocab-500: " + phase[1].split("] ")[1], "```"]
open(f"profiles/{tag}_kernels.md", "w").write("\n".join(txt) + "\n")
print("wrote", f"profiles/{tag}_sweep.md", f"profiles/{tag}_kernels.md")
