#!/bin/bash
# dense-merge validation: GPU tests touching the merge, torchrun both merges, merge cost table
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_engine.py tests/test_gpu_launcher.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/dense_tests.log 2>&1 || { tail -30 gpurun_out/dense_tests.log; exit 1; }
tail -3 gpurun_out/dense_tests.log
bash tools/dist_smoke.sh || exit 1
timeout -k 10 300 python tools/merge_cost.py 100000 1000000 > gpurun_out/merge_cost.md 2> gpurun_out/merge_cost.err || { tail gpurun_out/merge_cost.err; exit 1; }
cat gpurun_out/merge_cost.md
for m in shuffle dense; do
  WC_MERGE_ALWAYS=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 200)) bench.py --gpus 1 --steps 10 --warmup 2 \
    --vocab 1000000 --merge $m > gpurun_out/dist1m_$m.json 2> gpurun_out/dist1m_$m.err || { tail -20 gpurun_out/dist1m_$m.err; exit 1; }
  cut -c1-200 gpurun_out/dist1m_$m.json
done
