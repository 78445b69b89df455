#!/bin/bash
# bench.py at several vocabularies (no profiler), oracle-validated: tools/vocab_bench.sh [vocab ...]
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${@:-500 100000 1000000}; do
  timeout -k 10 180 python3 bench.py --vocab $v > gpurun_out/vb_$v.json 2> gpurun_out/vb_$v.err || { tail -5 gpurun_out/vb_$v.err; exit 1; }
  python3 -c "
import json,sys; d=[json.loads(l) for l in open('gpurun_out/vb_$v.json') if l.startswith('{')][-1]
print('vocab', $v, d['value'], 'GB/s', d['ms_per_step'], 'ms', 'validated', d['validated'], (d.get('validation') or {}).get('identical'))"
done
