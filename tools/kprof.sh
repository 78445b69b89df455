#!/bin/bash
# Per-kernel average times of any command (rocprofv3 kernel trace): tools/kprof.sh TAG cmd args...
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kp_$TAG -o run --output-format csv \
  -- "$@" > gpurun_out/kp_$TAG.log 2>&1 || { tail -5 gpurun_out/kp_$TAG.log; exit 1; }
python3 - gpurun_out/kp_$TAG "$TAG" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
print("==", sys.argv[2])
for r in rows[:24]:
    print("%-48s calls=%5s avg_us=%9.2f" % (r["Name"].split("(")[0][:48], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
grep -v '^\[\|^W2\|^E2' gpurun_out/kp_$TAG.log | tail -8
