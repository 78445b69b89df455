#!/bin/bash
# A/B: GPU tests, then bench with the current map kernel and the previous one (WC_MAP_V4=1).
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
timeout -k 10 120 python bench.py > gpurun_out/ab_new.json 2> gpurun_out/ab_new.err || exit 1
WC_MAP_V4=1 timeout -k 10 120 python bench.py > gpurun_out/ab_v4.json 2> gpurun_out/ab_v4.err || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof_ab.log 2>&1 || exit 1
python3 - <<'PY'
import json
for n in ("new","v4"):
    d=json.loads(open(f"gpurun_out/ab_{n}.json").read())
    print(n, d["value"], "GB/s", d["ms_per_step"], "ms", "records", d["stages"]["records"], "mr", d["stages"]["map_reduce_ms"], "fin", d["stages"]["finalize_ms"])
PY
