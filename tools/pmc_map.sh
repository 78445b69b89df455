#!/bin/bash
# PMC counters of the map / reduce kernels (each pass its own run; --pmc never combined with tracing).
export TMPDIR=/tmp
TAG=${1:-cur}; shift
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
for p in 1 2 3; do
  eval C=\$P$p
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'wc_map|wc_reduce' -d gpurun_out/pmc_${TAG}_$p -o run --output-format csv \
    -- python3 bench.py --steps 2 --warmup 0 "$@" > gpurun_out/pmc_${TAG}_$p.log 2>&1 || { echo "pass $p failed"; tail -3 gpurun_out/pmc_${TAG}_$p.log; exit 1; }
done
python3 - "$TAG" <<'PY'
import csv, collections, glob, sys
tag = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); nd = collections.defaultdict(set)
for f in glob.glob(f"gpurun_out/pmc_{tag}_*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = "map" if "wc_map" in r["Kernel_Name"] else "reduce"
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); nd[(k, f)].add(r["Dispatch_Id"])
for k, d in agg.items():
    n = max(len(v) for (kk, f), v in nd.items() if kk == k)
    print(k, " ".join(f"{c}={v/n:.3e}" for c, v in sorted(d.items())))
PY
