#!/bin/bash
# Host-side phases of ./wordcount FILE's streaming loop (WC_STREAM_TRACE=1:
# reads, launches, completion waits) on an 8 GiB synthetic file, warm page
# cache, for a few piece sizes -> gpurun_out/stream_trace.txt
export TMPDIR=/tmp
F=${WC_FILE_DIR:-/tmp}/wc_trace_8g.txt
OUT=gpurun_out/stream_trace.txt
mkdir -p gpurun_out
: > $OUT
timeout -k 10 300 python3 - "$F" <<'PY' || exit 1
import sys
from cuda_mapreduce_amd.ops import synth_host
with open(sys.argv[1], "wb") as f:
    for i in range(8):
        f.write(synth_host(1 << 30, first_segment=i * (1 << 20), seed=1, vocab=100000))
PY
timeout -k 10 120 cat $F > /dev/null || exit 1
for piece in 33554432 67108864 134217728; do
  for rep in 1 2; do
    WC_STREAM_TRACE=1 WC_STREAM_CHUNK=$piece timeout -k 10 300 ./wordcount $F --no-echo --no-list --bench-json /tmp/st.json > /dev/null 2> /tmp/st.err || { tail -3 /tmp/st.err; exit 1; }
    python3 -c "import json; d=json.load(open('/tmp/st.json')); print('piece %d MiB: %.2f GB/s streaming (%.3f s)' % ($piece >> 20, d['count_gb_per_s'], d['count_seconds']), end='  ')" >> $OUT
    grep "stream:" /tmp/st.err >> $OUT
  done
done
rm -f $F
cat $OUT
