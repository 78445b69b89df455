#!/bin/bash
# UTCL1 (per-CU TLB) translations and L2 read latency of the map / reduce kernels:
# tools/pmc_tlb.sh TAG [bench args]   (one --pmc pass of 4 TCP counters, no tracing)
export TMPDIR=/tmp
TAG=${1:-cur}; shift
C="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'wc_map|wc_reduce' -d gpurun_out/tlb_$TAG -o run --output-format csv \
  -- python3 bench.py --steps 2 --warmup 0 --no-oracle "$@" > gpurun_out/tlb_$TAG.log 2>&1 || { echo "pmc failed"; tail -3 gpurun_out/tlb_$TAG.log; exit 1; }
python3 - "$TAG" <<'PY'
import csv, collections, glob, sys
tag = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); nd = collections.defaultdict(set)
for f in glob.glob(f"gpurun_out/tlb_{tag}/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = "map" if "wc_map" in r["Kernel_Name"] else "reduce"
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); nd[k].add(r["Dispatch_Id"])
for k, d in agg.items():
    n = len(nd[k])
    print(tag, k, " ".join(f"{c}={v/n:.3e}" for c, v in sorted(d.items())))
PY
