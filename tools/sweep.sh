#!/bin/bash
# 1-GPU sweep of the BASELINE configs + vocabulary sizes -> gpurun_out/sweep.jsonl
export TMPDIR=/tmp
out=gpurun_out/sweep.jsonl; : > $out
run() { timeout -k 10 300 python bench.py "$@" 2>/dev/null | tail -1 >> $out || { echo "FAILED: $*"; exit 1; }; tail -1 $out | cut -c1-160; }
run --config 1gb --steps 10 --warmup 3
for v in 500 10000 1000000; do run --config 1gb --vocab $v --steps 10 --warmup 3; done
run --config 64gb --steps 2 --warmup 1
run --config 1tb-8gpu-host-staged --gb-per-gpu 16 --pool-gb 4 --steps 2 --warmup 1
