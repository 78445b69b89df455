#!/bin/bash
# shader clock of wc_map on this box: GRBM_GUI_ACTIVE (GPU busy cycles, summed over XCDs) per dispatch
# against the dispatch's duration, at v1m and v100k
export TMPDIR=/tmp
mkdir -p gpurun_out/clk
for v in 1000000 100000; do
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES --kernel-include-regex 'wc_map' -d gpurun_out/clk/v$v -o run --output-format csv \
    -- python3 bench.py --steps 10 --warmup 2 --no-oracle --vocab $v > gpurun_out/clk/v$v.log 2>&1 || { tail -3 gpurun_out/clk/v$v.log; exit 1; }
  python3 - $v <<'PY'
import csv, glob, sys, collections
v = sys.argv[1]
rows = list(csv.DictReader(open(glob.glob(f"gpurun_out/clk/v{v}/**/run_counter_collection.csv", recursive=True)[0])))
by = collections.defaultdict(dict)
for r in rows:
    by[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    by[r["Dispatch_Id"]]["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
xs = [d for d in by.values() if "GRBM_GUI_ACTIVE" in d][-5:]
for d in xs:
    print("v%s wc_map %.1f us, GRBM_GUI_ACTIVE %.3e (/8 XCDs -> %.2f GHz)" % (v, d["ns"] / 1e3, d["GRBM_GUI_ACTIVE"], d["GRBM_GUI_ACTIVE"] / 8 / d["ns"]))
PY
done
