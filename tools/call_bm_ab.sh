#!/bin/bash
# Reduce epilogue change: order / engine / exact / split-reduce GPU tests, then
# interleaved A/Bs at v1m and long30_v1m (and v100k), kernel stats at v1m.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_order.py tests/test_gpu_engine.py tests/test_gpu_exact.py tests/test_gpu_split_reduce.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bm_tests.log 2>&1 || { tail -20 gpurun_out/bm_tests.log; exit 1; }
tail -1 gpurun_out/bm_tests.log
for args in "--vocab 1000000" "--vocab 1000000 --long-frac 0.3" ""; do
  REPS=3 bash tools/vbench.sh $args || exit 1
done
bash tools/kstats_ab.sh --vocab 1000000 > gpurun_out/bm_ks.txt 2>&1 || exit 1
grep -E "==|wc_reduce|wc_bm|wc_map" gpurun_out/bm_ks.txt
bash tools/kstats_ab.sh > gpurun_out/bm_ks100k.txt 2>&1 || exit 1
grep -E "==|wc_fo" gpurun_out/bm_ks100k.txt
