#!/bin/bash
# insert-emit change: every merge GPU test, the merge tax of both builds (interleaved), W = 8 cost model
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_launcher.py tests/test_gpu_order.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ins_tests.log 2>&1 || { tail -20 gpurun_out/ins_tests.log; exit 1; }
tail -1 gpurun_out/ins_tests.log
for r in 1 2; do
  echo "== new"; REPS=1 bash tools/merge_tax.sh || exit 1
  echo "== base"; WC_LIB=$PWD/cuda_mapreduce_amd/lib/variants/libwc_base.so REPS=1 bash tools/merge_tax.sh || exit 1
done
bash tools/merge_rank_cost.sh 1 8 > gpurun_out/ins_mrc.txt 2>&1 || { tail gpurun_out/ins_mrc.txt; exit 1; }
grep -E "^\| (1|8) " gpurun_out/ins_mrc.txt
