#!/bin/bash
# Same-box sweep: decoupled (default) vs tile map kernel over vocabularies and the 64gb config.
export TMPDIR=/tmp
for args in "--vocab 100000" "--vocab 500" "--vocab 10000" "--vocab 1000000" "--config 64gb --steps 2 --warmup 1"; do
  for m in 1 0; do
    WC_MAP_DEC=$m timeout -k 10 200 python bench.py $args > gpurun_out/sw2.json 2>/dev/null || { echo "FAILED $args $m"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/sw2.json').read()); print('%-40s dec=$m %8.1f GB/s records %.1fM' % ('$args', d['value'], d['stages']['records']/1e6))"
  done
done
