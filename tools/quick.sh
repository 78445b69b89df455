#!/bin/bash
# quick perf check: GPU tests (subset) + bench + phase clock
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "not loopback" > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
timeout -k 10 120 python bench.py > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/q_bench.json').read()); st=d['stages']
print(d['value'],'GB/s', d['ms_per_step'],'ms  mr',st['map_reduce_ms'],'fin',st['finalize_ms'],'records',st['records'])"
WC_MAP_STAMPS=1 timeout -k 10 120 python bench.py --steps 3 --warmup 1 2>&1 | grep "phase clock"
timeout -k 10 120 python bench.py --vocab 500 > gpurun_out/q_bench500.json 2>/dev/null || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/q_bench500.json').read()); print('vocab500', d['value'],'GB/s')"
