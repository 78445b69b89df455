#!/bin/bash
# Merge changes: GPU engine tests (loopback + RCCL-at-world-1 merges), merge tax, step timelines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_launcher.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/merge_tests.log 2>&1 || { tail -20 gpurun_out/merge_tests.log; exit 1; }
tail -1 gpurun_out/merge_tests.log
REPS=${REPS:-2} bash tools/merge_tax.sh || exit 1
bash tools/step_timelines.sh > gpurun_out/step_timelines.txt 2>&1 || { tail gpurun_out/step_timelines.txt; exit 1; }
grep -E "==|merge|owner|mrow|step span" gpurun_out/step_timelines.txt
