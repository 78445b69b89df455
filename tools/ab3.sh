#!/bin/bash
export TMPDIR=/tmp
for m in ${MODES:-0 7 0 7}; do
  WC_ABLATE_MAP=$m timeout -k 10 120 python bench.py > gpurun_out/ab3.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab3.json').read()); print('mode $m', d['value'], d['ms_per_step'], d['stages']['records'])"
done
WC_ABLATE_MAP=7 WC_MAP_STAMPS=1 timeout -k 10 120 python bench.py --steps 3 --warmup 1 2>&1 | grep "phase clock"
