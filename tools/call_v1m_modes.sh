#!/bin/bash
# v1m process bimodality: 6 fresh processes of the v1m bench,
# then 4 processes each with one UTCL1 / L2-latency PMC pass (tools/pmc_tlb.sh)
# and 4 with one HBM-bytes pass, each tagged with its own GB/s.
export TMPDIR=/tmp
mkdir -p gpurun_out/v1m_modes
for i in 1 2 3 4 5 6; do
  timeout -k 10 120 python3 bench.py --vocab 1000000 --steps 100 --warmup 10 --no-oracle > gpurun_out/v1m_modes/b$i.json 2> /dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/v1m_modes/b$i.json').read().strip().splitlines()[-1]); print('proc $i', d['value'], d['stages']['device_ms'])"
done
for i in 1 2 3 4; do
  bash tools/pmc_tlb.sh v1m_$i --vocab 1000000 || exit 1
done
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum"
for i in 1 2 3 4; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'wc_map|wc_reduce' -d gpurun_out/v1m_modes/l2_$i -o run --output-format csv \
    -- python3 bench.py --steps 2 --warmup 0 --no-oracle --vocab 1000000 > gpurun_out/v1m_modes/l2_$i.log 2>&1 || { tail -3 gpurun_out/v1m_modes/l2_$i.log; exit 1; }
  python3 - $i <<'PY'
import csv, collections, glob, sys
i = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); nd = collections.defaultdict(set)
for f in glob.glob(f"gpurun_out/v1m_modes/l2_{i}/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = "map" if "wc_map" in r["Kernel_Name"] else "reduce"
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); nd[k].add(r["Dispatch_Id"])
for k, d in agg.items():
    n = len(nd[k])
    print("l2", i, k, " ".join(f"{c}={v/n:.3e}" for c, v in sorted(d.items())))
PY
done
