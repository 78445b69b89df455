#!/bin/bash
# Per-kernel mean times over many steps for the default build and every variant
# library, interleaved REPS times (rocprofv3 kernel trace): tools/kstats_long.sh [bench args]
export TMPDIR=/tmp
REPS=${REPS:-2}
libs="cuda_mapreduce_amd/lib/libwc.so $(ls cuda_mapreduce_amd/lib/variants/*.so 2>/dev/null)"
for r in $(seq $REPS); do
  for so in $libs; do
    n=$(basename $so .so)
    WC_LIB=$PWD/$so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kl_${n}_$r -o run --output-format csv \
      -- python3 bench.py --steps 60 --warmup 20 --no-oracle "$@" > gpurun_out/kl_${n}_$r.log 2>&1 || { echo "FAILED $n"; exit 1; }
    python3 - gpurun_out/kl_${n}_$r "$n" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
rows = {r["Name"].split("(")[0].replace("void ", "").replace("wc::dev::", ""): r for r in csv.DictReader(open(f))}
keep = ["wc_map<false, false>", "wc_map<false, true>", "wc_map<false>", "wc_reduce_buckets<false>", "wc_reduce_buckets<true>",
        "wc_reduce_buckets", "wc_hot_sample", "wc_hot_merge", "wc_fo_bin", "wc_fo_sort", "wc_publish"]
print("%-14s " % sys.argv[2] + " ".join("%s=%.1f" % (k.replace("wc_", ""), float(rows[k]["AverageNs"]) / 1e3) for k in keep if k in rows))
PY
  done
done
