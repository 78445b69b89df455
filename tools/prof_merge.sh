#!/bin/bash
# kernel trace of the merge protocols (tools/merge_cost.py) + PMC passes of the shipped map/reduce
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pm -o run --output-format csv \
  -- python3 tools/merge_cost.py ${VOCABS:-100000 1000000} > gpurun_out/pm.log 2>&1 || { tail -5 gpurun_out/pm.log; exit 1; }
f=$(find gpurun_out/pm -name 'run_kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:30]:
    print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>6s} avg_us={float(r["AverageNs"])/1e3:9.2f} tot_ms={float(r["TotalDurationNs"])/1e6:9.2f}')
PY
