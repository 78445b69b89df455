#!/bin/bash
# v1m box check: one bench; on a slow-mode box (< 780 GB/s) the same PMC passes
# as tools/call_v1m_modes.sh plus an HBM write-request pass, for comparison with
# the fast-mode counters in profiles/r6_v1m/modes_and_pmc.txt.
export TMPDIR=/tmp
mkdir -p gpurun_out/v1m_slow
timeout -k 10 120 python3 bench.py --vocab 1000000 --steps 100 --warmup 10 --no-oracle > gpurun_out/v1m_slow/b.json 2> /dev/null || exit 1
v=$(python3 -c "import json; d=json.loads(open('gpurun_out/v1m_slow/b.json').read().strip().splitlines()[-1]); print(d['value'])")
python3 -c "import json; d=json.loads(open('gpurun_out/v1m_slow/b.json').read().strip().splitlines()[-1]); print('v1m', d['value'], d['stages']['device_ms'])"
python3 -c "import sys; sys.exit(0 if float('$v') < 780 else 1)" || { echo "fast box: no PMC"; exit 0; }
bash tools/pmc_tlb.sh v1m_slow --vocab 1000000 || exit 1
for C in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  tag=$(echo $C | cut -c1-12 | tr ' ' _)
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'wc_map|wc_reduce' -d gpurun_out/v1m_slow/$tag -o run --output-format csv \
    -- python3 bench.py --steps 2 --warmup 0 --no-oracle --vocab 1000000 > gpurun_out/v1m_slow/$tag.log 2>&1 || { tail -3 gpurun_out/v1m_slow/$tag.log; exit 1; }
  python3 - $tag <<'PY'
import csv, collections, glob, sys
t = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); nd = collections.defaultdict(set)
for f in glob.glob(f"gpurun_out/v1m_slow/{t}/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = "map" if "wc_map" in r["Kernel_Name"] else "reduce"
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); nd[k].add(r["Dispatch_Id"])
for k, d in agg.items():
    n = len(nd[k])
    print(t, k, " ".join(f"{c}={v/n:.3e}" for c, v in sorted(d.items())))
PY
done
