#!/bin/bash
# quick perf check: GPU tests + bench + map phase clock + vocabulary 500 / 1M benches
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${QK:+-k "$QK"} > gpurun_out/q_tests.log 2>&1 || { tail -40 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
for v in 100000 500 1000000; do
  timeout -k 10 120 python bench.py --vocab $v > gpurun_out/q_bench_$v.json 2> gpurun_out/q_bench_$v.err || { tail -5 gpurun_out/q_bench_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/q_bench_$v.json').read()); st=d['stages']
print('vocab $v:', d['value'],'GB/s', d['ms_per_step'],'ms  device',st['device_ms'],'records',st['records'],'valid',d['validated'])"
done
WC_MAP_STAMPS=1 timeout -k 10 120 python bench.py --steps 3 --warmup 1 2>&1 | grep "phase clock"
