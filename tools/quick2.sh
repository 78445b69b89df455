#!/bin/bash
# GPU tests (both map kernels) + bench both + phase clock
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q2_tests.log 2>&1 || { tail -30 gpurun_out/q2_tests.log; exit 1; }
tail -1 gpurun_out/q2_tests.log
WC_MAP_DEC=0 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "not loopback" > gpurun_out/q2_tests0.log 2>&1 || { tail -30 gpurun_out/q2_tests0.log; exit 1; }
tail -1 gpurun_out/q2_tests0.log
for m in 1 0; do for v in 100000 500; do
  WC_MAP_DEC=$m timeout -k 10 120 python bench.py --vocab $v > gpurun_out/q2.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/q2.json').read()); st=d['stages']; print('dec=$m vocab=$v', d['value'], 'GB/s', d['ms_per_step'], 'ms mr', st['map_reduce_ms'], 'fin', st['finalize_ms'], 'records', st['records'])"
done; done
WC_MAP_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 2>&1 | grep "phase clock"
