#!/bin/bash
# LDS bank-conflict share of the reduce's random-slot access pattern vs
# conflict-free baselines (tools/probe/lds_conflicts.hip), one counter pass.
#   tools/lds_probe.sh -> gpurun_out/lds_probe/ + summary on stdout
export TMPDIR=/tmp
mkdir -p gpurun_out/lds_probe
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES \
  -d gpurun_out/lds_probe -o run --output-format csv -- tools/probe/lds_conflicts > gpurun_out/lds_probe/log.txt 2>&1 || { tail -5 gpurun_out/lds_probe/log.txt; exit 1; }
grep "mode" gpurun_out/lds_probe/log.txt
python3 - <<'PY'
import csv, collections, glob
f = glob.glob("gpurun_out/lds_probe/**/run_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    if "k_probe" not in k:
        continue
    print("%-40s conflict share %.3f  (bank conflict %.3e / idx active %.3e, LDS instrs %.3e)" % (
        k, d["SQ_LDS_BANK_CONFLICT"] / max(1, d["SQ_LDS_IDX_ACTIVE"]), d["SQ_LDS_BANK_CONFLICT"],
        d["SQ_LDS_IDX_ACTIVE"], d["SQ_INSTS_LDS"]))
PY
