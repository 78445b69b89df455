#!/bin/bash
# File-path streaming piece sweep: 4 GiB synthetic file through ./wordcount (pinned ring = 3 pieces).
export TMPDIR=/tmp
F=/tmp/wc_fsweep_4g.txt
timeout -k 10 120 python3 - "$F" <<'PY' || exit 1
import sys
from cuda_mapreduce_amd.ops import synth_host
with open(sys.argv[1], "wb") as f:
    for i in range(4):
        f.write(synth_host(1 << 30, first_segment=i * (1 << 20), seed=1, vocab=100000))
PY
for c in 268435456 67108864 33554432 16777216 8388608 default; do
  if [ $c = default ]; then unset WC_STREAM_CHUNK; else export WC_STREAM_CHUNK=$c; fi
  timeout -k 10 120 ./wordcount $F --no-echo --no-list --bench-json /tmp/b.json > /dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('/tmp/b.json')); print('piece %-10s %6.2f GB/s  %.3f s  map+reduce %.0f ms  chunks %d tokens %d' % (sys.argv[1], d['gb_per_s'], d['seconds'], d['device_ms']['map'] + d['device_ms']['reduce'], d['chunks'], d['tokens']))" $c
done | tee gpurun_out/file_chunk_sweep.txt
unset WC_STREAM_CHUNK
WC_IO_THREADS=16 timeout -k 10 120 ./wordcount $F --no-echo --no-list --bench-json /tmp/b.json > /dev/null || exit 1
python3 -c "import json; d=json.load(open('/tmp/b.json')); print('default, 16 read threads %6.2f GB/s  %.3f s  map+reduce %.0f ms' % (d['gb_per_s'], d['seconds'], d['device_ms']['map'] + d['device_ms']['reduce']))" | tee -a gpurun_out/file_chunk_sweep.txt
rm -f $F
