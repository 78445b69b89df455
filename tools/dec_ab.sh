#!/bin/bash
export TMPDIR=/tmp
WC_MAP_DEC=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dec_tests.log 2>&1 || { tail -30 gpurun_out/dec_tests.log; exit 1; }
tail -1 gpurun_out/dec_tests.log
for m in 0 1 0 1; do
  WC_MAP_DEC=$m timeout -k 10 120 python bench.py > gpurun_out/dec.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/dec.json').read()); print('dec=$m', d['value'], d['ms_per_step'], d['stages']['records'])"
done
WC_MAP_DEC=1 timeout -k 10 120 python bench.py --vocab 500 > gpurun_out/dec.json 2>/dev/null && python3 -c "import json; d=json.loads(open('gpurun_out/dec.json').read()); print('dec=1 vocab500', d['value'])"
WC_MAP_DEC=1 WC_MAP_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 2>&1 | grep "phase clock"
