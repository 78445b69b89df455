#!/bin/bash
# XCD-weighted map ranges A/B: GPU engine/exact tests on the new build, validated
# bench, interleaved A/B against the variants, per-XCD map block durations.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_exact.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/xw_tests.log 2>&1 || { tail -20 gpurun_out/xw_tests.log; exit 1; }
tail -1 gpurun_out/xw_tests.log
timeout -k 10 200 python3 bench.py --steps 100 --warmup 10 > gpurun_out/xw_bench.json 2> gpurun_out/xw_bench.err || { tail -5 gpurun_out/xw_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/xw_bench.json').read().strip().splitlines()[-1]); print('validated bench', d['value'], d['validated'], d['stages']['device_ms'])"
REPS=${REPS:-3} bash tools/vbench.sh || exit 1
for x in 1 0; do
WC_MAP_XW=$x WC_MAP_STAMPS=1 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-oracle > /dev/null 2> gpurun_out/xw_stamps_$x.err || exit 1
echo "WC_MAP_XW=$x"; grep -E "map blocks|xcc" gpurun_out/xw_stamps_$x.err
done
