#!/bin/bash
# The `./wordcount <file>` path (north-star form) on one MI355X:
#  1. a 16 GiB synthetic file (Zipf(1.0), 100k words) written to $WC_FILE_DIR
#     (default /tmp) and read once (warm page cache);
#  2. the raw host read rate of the same reader (pread_parallel into pinned
#     memory, no GPU copy) and pinned H2D from the GPU's own NUMA node and
#     from every other node;
#  3. ./wordcount FILE --no-echo --no-list twice (GB/s = file bytes / CLI wall
#     time, HIP start-up included);
#  4. a 1 GiB file: GPU output byte-identical to --cpu.
# -> gpurun_out/file_path.txt
export TMPDIR=/tmp
D=${WC_FILE_DIR:-/tmp}
F=$D/wc_file_16g.txt
G=$D/wc_file_1g.txt
mkdir -p gpurun_out
OUT=gpurun_out/file_path.txt
: > $OUT
timeout -k 10 300 python3 - "$F" "$G" <<'PY' || exit 1
import sys
from cuda_mapreduce_amd.ops import synth_host
with open(sys.argv[1], "wb") as f:
    for i in range(16):
        f.write(synth_host(1 << 30, first_segment=i * (1 << 20), seed=1, vocab=100000))
        print("wrote GiB", i + 1, flush=True)
with open(sys.argv[2], "wb") as f:
    f.write(synth_host(1 << 30, first_segment=0, seed=3, vocab=100000))
PY
timeout -k 10 120 cat $F > /dev/null || exit 1
timeout -k 10 300 python3 - "$F" >> $OUT <<'PY' || exit 1
import glob, sys
from cuda_mapreduce_amd import ops
for piece in (64 << 20, 256 << 20):
    g, n = ops.file_read_bench(sys.argv[1], piece=piece)
    print("raw read (pread_parallel -> pinned, node-bound), piece %d MiB: %.2f GB/s over %.1f GiB" % (piece >> 20, g, n / 2**30))
nodes = sorted(int(p.split("node")[-1]) for p in glob.glob("/sys/devices/system/node/node[0-9]*"))
g, used = ops.h2d_bench(0, -1, 1 << 30, 8)
print("pinned H2D from the GPU's node (%d): %.2f GB/s" % (used, g))
for nd in nodes:
    g, used = ops.h2d_bench(0, nd, 1 << 30, 8)
    print("pinned H2D from node %d: %.2f GB/s (bound: %s)" % (nd, g, used >= 0))
PY
for piece in 67108864 268435456 67108864 268435456; do
  WC_STREAM_CHUNK=$piece timeout -k 10 300 ./wordcount $F --no-echo --no-list --bench-json /tmp/fp.json > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('/tmp/fp.json')); print('wordcount 16 GiB file, %d MiB pieces: %.2f GB/s wall (%.3f s, HIP + engine start-up included), %.2f GB/s streaming (%.3f s in count)  map %.0f ms reduce %.0f ms  chunks %d  tokens %d' % ($piece >> 20, d['gb_per_s'], d['seconds'], d['count_gb_per_s'], d['count_seconds'], d['device_ms']['map'], d['device_ms']['reduce'], d['chunks'], d['tokens']))" >> $OUT
done
timeout -k 10 300 ./wordcount $G --no-echo > /tmp/fp_gpu.txt || exit 1
timeout -k 10 300 ./wordcount $G --no-echo --cpu > /tmp/fp_cpu.txt || exit 1
if cmp -s /tmp/fp_gpu.txt /tmp/fp_cpu.txt; then echo "1 GiB file: GPU output identical to --cpu ($(wc -l < /tmp/fp_cpu.txt) lines)" >> $OUT;
else echo "1 GiB file: GPU output DIFFERS from --cpu" >> $OUT; fi
rm -f $F $G
cat $OUT
