#!/bin/bash
# Per-variant kernel times (rocprofv3 --kernel-trace --stats) of the default build and every
# variant in cuda_mapreduce_amd/lib/variants: tools/vprof.sh [bench args]
export TMPDIR=/tmp
for so in cuda_mapreduce_amd/lib/libwc.so cuda_mapreduce_amd/lib/variants/*.so; do
  [ -f "$so" ] || continue
  n=$(basename $so .so)
  WC_LIB=$PWD/$so timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/vp_$n -o run --output-format csv \
    -- python3 bench.py --steps 5 --warmup 1 "$@" > gpurun_out/vp_$n.log 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FAILED $so rc=$rc"; tail -3 gpurun_out/vp_$n.log; exit 1; fi
  python3 - gpurun_out/vp_$n "$n" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    nm = r["Name"]
    for k in ("wc_map", "wc_reduce", "wc_fo_bin", "wc_fo_sort"):
        if k in nm:
            out.append("%s %.1f us" % (k, float(r["AverageNs"]) / 1e3))
print("%-12s %s" % (sys.argv[2], "  ".join(out)))
PY
done
