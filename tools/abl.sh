#!/bin/bash
# Map ablations for the current kernel (and v4 if V4=1): kernel time of wc_map_tokenize per mode.
export TMPDIR=/tmp
for m in ${MODES:-1 2 5}; do
  WC_ABLATE_MAP=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/abl$m -o run --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/abl$m.log 2>&1 || exit 1
  echo "mode $m: $(grep wc_map_tokenize gpurun_out/abl$m/run_kernel_stats.csv | cut -d, -f2-5)"
done
