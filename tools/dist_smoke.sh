#!/bin/bash
# torch.distributed.run launcher path of bench.py at --nproc-per-node 1 with the
# RCCL communicator forced on (WC_MERGE_ALWAYS=1), once per merge protocol.
export TMPDIR=/tmp
for m in shuffle dense; do
  WC_MERGE_ALWAYS=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 200)) bench.py --gpus 1 --steps 10 --warmup 2 \
    --merge $m > gpurun_out/dist_$m.json 2> gpurun_out/dist_$m.err || { tail -20 gpurun_out/dist_$m.err; exit 1; }
  cut -c1-300 gpurun_out/dist_$m.json
done
