#!/bin/bash
# Round-3 check: kernel unit tests first (short limit), GPU tests, driver-style bench,
# RCCL merge forced at world 1 (both protocols).
export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest tests/test_gpu_engine.py -k radix -x -q --timeout 60 --timeout-method thread \
  > gpurun_out/r3_sort.log 2>&1
rc=$?; tail -3 gpurun_out/r3_sort.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${1:+-k "$1"} \
  > gpurun_out/r3_gtest.log 2>&1
rc=$?; tail -15 gpurun_out/r3_gtest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --steps 200 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || exit 1
cut -c1-900 gpurun_out/r3_bench.json
for m in shuffle dense; do
  WC_MERGE_ALWAYS=1 timeout -k 10 120 python bench.py --steps 200 --merge $m > gpurun_out/r3_merge_$m.json \
    2> gpurun_out/r3_merge_$m.err || { tail -20 gpurun_out/r3_merge_$m.err; exit 1; }
  cut -c1-900 gpurun_out/r3_merge_$m.json
done
