#!/bin/bash
# Checkpoint overhead and raw PCIe H2D ceiling on one MI355X (writes gpurun_out/ckpt_cost.txt):
#   - a 4 GiB synthetic file (Zipf-100k) counted by ./wordcount from disk (pread -> pinned ring -> GPU)
#     plain vs --checkpoint every 1 GiB / 256 MiB, and a crash after 2 checkpoints + --resume
#   - pinned host -> device hipMemcpy bandwidth (torch), the bound of every host-staged path
export TMPDIR=/tmp
set -o pipefail
OUT=gpurun_out/ckpt_cost.txt
F=/tmp/wc_ckpt_4g.txt
timeout -k 10 120 python3 - "$F" <<'EOF' || exit 1
import sys
from cuda_mapreduce_amd.ops import synth_host
with open(sys.argv[1], "wb") as f:
    for i in range(4):   # 4 x 1 GiB, segment-addressed so the file is one continuous stream
        f.write(synth_host(1 << 30, first_segment=i * (1 << 20), seed=1, vocab=100000))
EOF
: > $OUT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 180 ./wordcount $F --no-echo --no-list --bench-json /tmp/b.json "$@" > /tmp/w.out || return 1
  python3 -c "import json,sys; d=json.load(open('/tmp/b.json')); print('%-34s %7.2f GB/s  %.3f s (map+reduce %.0f ms, finalize %.0f ms, %d chunks)  tokens %d keys %d  total=%s' % (sys.argv[1], d['gb_per_s'], d['seconds'], d['device_ms']['map'] + d['device_ms']['reduce'], d['device_ms']['finalize'], d['chunks'], d['tokens'], d['keys'], open('/tmp/w.out').read().split('Total Count:')[1].strip()))" "$name" >> $OUT
}
WC_IO_THREADS=1 run "plain, 1 read thread" && \
run "plain (file -> pinned ring)" && \
run "checkpoint every 1 GiB" --checkpoint /tmp/ck1 --checkpoint-every 1G && \
run "checkpoint every 256 MiB" --checkpoint /tmp/ck2 --checkpoint-every 256M || { cat $OUT; exit 1; }
WC_CKPT_STOP_AFTER=2 timeout -k 10 180 ./wordcount $F --no-echo --no-list --checkpoint /tmp/ck3 --checkpoint-every 1G > /dev/null 2>&1
[ $? -eq 1 ] || { echo "crash injection did not stop the run" >> $OUT; cat $OUT; exit 1; }
run "resume after crash at 2 of 4 GiB" --checkpoint /tmp/ck3 --checkpoint-every 1G --resume || { cat $OUT; exit 1; }
timeout -k 10 120 python3 - >> $OUT <<'EOF' || exit 1
import time, torch
n = 1 << 30
h = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device="cuda")
for _ in range(3):
    d.copy_(h, non_blocking=True)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    d.copy_(h, non_blocking=True)
torch.cuda.synchronize()
print("pinned H2D hipMemcpy (1 GiB x10): %.2f GB/s" % (10 * n / (time.perf_counter() - t) / 1e9))
EOF
rm -f $F /tmp/ck1 /tmp/ck2 /tmp/ck3
cat $OUT
