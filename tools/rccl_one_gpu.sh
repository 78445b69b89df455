#!/bin/bash
# Two RCCL ranks on ONE GPU: both rank
# processes get LOCAL_RANK=0, share rank 0's RCCL id through the job's file
# rendezvous and run bench.py with the merge on (world size 2).  Either RCCL
# accepts the duplicate device — then this is a real two-rank RCCL run of the
# merge (grouped send / recv, reduce-scatter, all-gather) on one card — or it
# refuses, and the rank's stderr holds RCCL's exact message.
#   tools/rccl_one_gpu.sh [bench args]   -> gpurun_out/rccl1g_rank{0,1}.{out,err}
export TMPDIR=/tmp
mkdir -p gpurun_out
rdzv=$(mktemp -d /tmp/wc_rdzv_dup_XXXX)
port=$(python3 -c 'import socket; s=socket.socket(); s.bind(("127.0.0.1",0)); print(s.getsockname()[1])')
pids=()
for r in 0 1; do
  RANK=$r LOCAL_RANK=0 WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
  WC_RDZV_DIR=$rdzv WC_COMM_TIMEOUT_S=60 HSA_ENABLE_IPC_MODE_LEGACY=0 NCCL_DEBUG=${NCCL_DEBUG:-WARN} \
    timeout -k 10 150 python3 bench.py --gpus 2 "$@" > gpurun_out/rccl1g_rank$r.out 2> gpurun_out/rccl1g_rank$r.err &
  pids+=($!)
done
rc=0
for i in 0 1; do
  wait ${pids[$i]}; c=$?
  echo "rank $i exit $c"
  [ $c -ne 0 ] && rc=$c
done
rm -rf $rdzv
for r in 0 1; do echo "== rank $r stdout"; tail -c 3000 gpurun_out/rccl1g_rank$r.out; echo "== rank $r stderr"; tail -40 gpurun_out/rccl1g_rank$r.err; done
exit $rc
