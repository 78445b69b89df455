#!/bin/bash
# map-kernel changes: engine / exact GPU tests, the steady-state interleaved
# A/B (tools/call_long_ab.sh), then kernel stats of both builds
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_exact.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/map_tests.log 2>&1 || { tail -20 gpurun_out/map_tests.log; exit 1; }
tail -1 gpurun_out/map_tests.log
timeout -k 10 900 bash tools/call_long_ab.sh "$@" > gpurun_out/map_ab.txt 2>&1 || { tail -20 gpurun_out/map_ab.txt; exit 1; }
tail -3 gpurun_out/map_ab.txt
