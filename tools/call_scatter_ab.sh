#!/bin/bash
# owner-scatter change: every merge GPU test, the merge tax of both builds
# (interleaved, two rounds), and the merge kernels' times of each build
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_launcher.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sc_tests.log 2>&1 || { tail -20 gpurun_out/sc_tests.log; exit 1; }
tail -1 gpurun_out/sc_tests.log
for r in 1 2; do
  echo "== new"; REPS=1 bash tools/merge_tax.sh || exit 1
  echo "== base"; WC_LIB=$PWD/cuda_mapreduce_amd/lib/variants/libwc_base.so REPS=1 bash tools/merge_tax.sh || exit 1
done
for so in cuda_mapreduce_amd/lib/libwc.so cuda_mapreduce_amd/lib/variants/libwc_base.so; do
  n=$(basename $so .so)
  WC_LIB=$PWD/$so WC_MERGE_ALWAYS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sc_$n -o run --output-format csv \
    -- python3 bench.py --steps 10 --warmup 2 --no-oracle > gpurun_out/sc_$n.log 2>&1 || exit 1
  python3 - gpurun_out/sc_$n $n <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("insert_emit", "owner_scatter", "regions_to_cols")):
        print("%-12s %-40s avg_us=%8.2f" % (sys.argv[2], r["Name"].split("(")[0][:40], float(r["AverageNs"]) / 1e3))
PY
done
