#!/bin/bash
# One PMC pass (instruction mix) per engine build: the default libwc.so and every
# cuda_mapreduce_amd/lib/variants/*.so (tools/variants.sh), wc_map kernels only.
export TMPDIR=/tmp
C=${PMC:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"}
for so in cuda_mapreduce_amd/lib/libwc.so cuda_mapreduce_amd/lib/variants/*.so; do
  [ -f "$so" ] || continue
  n=$(basename $so .so)
  WC_LIB=$PWD/$so timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex 'wc_map' -d gpurun_out/pv_$n -o run \
    --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-oracle "$@" > gpurun_out/pv_$n.log 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FAILED $so rc=$rc"; tail -3 gpurun_out/pv_$n.log; exit 1; fi
  python3 - gpurun_out/pv_$n "$n" <<'PY'
import csv, collections, glob, sys
agg = collections.defaultdict(float); ds = set()
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wc_map" not in r["Kernel_Name"]: continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); ds.add(r["Dispatch_Id"])
n = max(len(ds), 1)
print("%-14s %s" % (sys.argv[2], " ".join("%s=%.3e" % (c.replace("SQ_", ""), v / n) for c, v in sorted(agg.items()))))
PY
done
