#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 120 python bench.py > gpurun_out/ab_new.json 2> gpurun_out/ab_new.err || exit 1
WC_MAP_V4=1 timeout -k 10 120 python bench.py > gpurun_out/ab_v4.json 2> gpurun_out/ab_v4.err || exit 1
python3 - <<'PY'
import json
for n in ("new","v4"):
    d=json.loads(open(f"gpurun_out/ab_{n}.json").read())
    print(n, d["value"], "GB/s", d["ms_per_step"], "ms", "records", d["stages"]["records"], "mr", d["stages"]["map_reduce_ms"], "fin", d["stages"]["finalize_ms"])
PY
MODES="1 2" bash tools/abl.sh
