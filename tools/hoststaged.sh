#!/bin/bash
# host-staged config on one GPU: native pinned pool (build time, peak RSS) + replay over PCIe, oracle-validated
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config 1tb-8gpu-host-staged --gpus 1 --gb-per-gpu ${GB:-16} --steps 2 --warmup 1 \
  > gpurun_out/hs.json 2> gpurun_out/hs.err || { tail -5 gpurun_out/hs.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/hs.json').read())
print('host-staged', d['value'], 'GB/s', d['ms_per_step'], 'ms valid', d['validated'], d.get('validation'), d.get('host_pool'))"
