#!/bin/bash
export TMPDIR=/tmp
for m in 0 5 3; do
  WC_ABLATE_MAP=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ab5_$m -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/ab5_$m.log 2>&1 || exit 1
  echo "mode $m: $(grep wc_map gpurun_out/ab5_$m/run_kernel_stats.csv | cut -d, -f2-4)"
done
