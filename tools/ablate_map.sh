#!/bin/bash
# Map-kernel ablations (MapArgs::ablate via WC_ABLATE_MAP), one rocprofv3 run each.
#   0 full | 1 keys only | 2 scan only | 3 no directory stores | 5 flush = clear only | 6 no count/min atomics
export TMPDIR=/tmp
for m in ${MODES:-0 1 2 3 4}; do
  WC_ABLATE_MAP=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/abl$m -o run --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/abl$m.log 2>&1 || exit 1
done
