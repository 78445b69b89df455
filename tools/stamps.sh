#!/bin/bash
# map phase clock + slow-path counters (diagnostic build path, WC_MAP_STAMPS=1)
export TMPDIR=/tmp
for v in 100000 ${VOCABS}; do
  WC_MAP_STAMPS=1 timeout -k 10 120 python bench.py --steps 3 --warmup 1 --vocab $v 2>&1 | grep "phase clock" | sed "s/^/vocab $v: /"
done
