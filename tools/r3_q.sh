#!/bin/bash
# Quick round-3 check: sort + exactness tests, then the headline bench, the LONG-word load and a kernel trace.
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_engine.py -k "order or radix or golden or loopback_merge_speculative" -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r3q_t1.log 2>&1
rc=$?; tail -2 gpurun_out/r3q_t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3q_t2.log 2>&1
rc=$?; tail -2 gpurun_out/r3q_t2.log; [ $rc -eq 0 ] || exit $rc
bash tools/r3_sweep.sh v100k v1m long30_v1m || exit 1
bash tools/kstats.sh cur || exit 1
bash tools/kstats.sh v1m --vocab 1000000 || exit 1
bash tools/kstats.sh long30 --vocab 1000000 --long-frac 0.3
