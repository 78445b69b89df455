#!/bin/bash
# Round-end validation of the shipped build: the whole GPU suite, the default
# bench (validated), kernel statistics at v100k and v1m, step timelines.
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/gtest.log 2>&1 || { tail -20 gpurun_out/final/gtest.log; exit 1; }
tail -1 gpurun_out/final/gtest.log
timeout -k 10 300 python3 bench.py > gpurun_out/final/bench_default.json 2> gpurun_out/final/bench_default.err || { tail -5 gpurun_out/final/bench_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/final/bench_default.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['steps'], d['validated'], d['stages']['device_ms'])"
bash tools/kstats.sh final_v100k > gpurun_out/final/kstats_v100k.txt 2>&1 || exit 1
bash tools/kstats.sh final_v1m --vocab 1000000 > gpurun_out/final/kstats_v1m.txt 2>&1 || exit 1
head -12 gpurun_out/final/kstats_v100k.txt
bash tools/step_timelines.sh > gpurun_out/final/step_timelines.txt 2>&1 || exit 1
grep -E "==|step span" gpurun_out/final/step_timelines.txt
