#!/bin/bash
# Kernel times vs vocabulary size (combiner hit rate), one rocprofv3 run each.
export TMPDIR=/tmp
for v in ${VOCABS:-500 10000 100000 1000000}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/voc$v -o run --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 --vocab $v > gpurun_out/voc$v.log 2>&1 || exit 1
done
