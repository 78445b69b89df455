#!/bin/bash
# wc_mrow_insert_emit ablations (profiling builds, results invalid): kernel time
# of the shipped build vs no row-index atomic (ie1), + no CAS (ie2), + no count atomics (ie3)
export TMPDIR=/tmp
mkdir -p gpurun_out/ie
for so in cuda_mapreduce_amd/lib/libwc.so cuda_mapreduce_amd/lib/variants/libwc_ie*.so; do
  n=$(basename $so .so)
  WC_LIB=$PWD/$so WC_MERGE_ALWAYS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ie/$n -o run --output-format csv \
    -- python3 bench.py --steps 10 --warmup 2 --no-oracle > gpurun_out/ie/$n.log 2>&1
  rc=$?; [ $rc -le 1 ] || { echo "$n rc=$rc"; tail -3 gpurun_out/ie/$n.log; exit 1; }
  python3 - gpurun_out/ie/$n $n <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("insert_emit", "owner_scatter", "regions_to_cols")):
        print("%-10s %-40s calls=%4s avg_us=%8.2f" % (sys.argv[2], r["Name"].split("(")[0][:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
