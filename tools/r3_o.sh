#!/bin/bash
# First-occurrence order check: order tests, the sort microbench (+ per-kernel trace), kernel traces at 100k and 1M keys.
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_order.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3o_t.log 2>&1
rc=$?; tail -3 gpurun_out/r3o_t.log; [ $rc -eq 0 ] || exit $rc
bash tools/kprof.sh sort python3 tools/sort_bench.py || exit 1
bash tools/kstats.sh cur || exit 1
bash tools/kstats.sh v1m --vocab 1000000
