#!/bin/bash
# Kernel + memory-copy trace of the file-streaming CLI path (4 GiB synthetic file, 64 MiB pieces):
# shows the H2D copies overlapping the map/reduce kernels.  -> gpurun_out/prof_file/, summary on stdout
export TMPDIR=/tmp
F=/tmp/wc_prof_4g.txt
timeout -k 10 120 python3 - "$F" <<'PY' || exit 1
import sys
from cuda_mapreduce_amd.ops import synth_host
with open(sys.argv[1], "wb") as f:
    for i in range(4):
        f.write(synth_host(1 << 30, first_segment=i * (1 << 20), seed=1, vocab=100000))
PY
./wordcount $F --no-echo --no-list > /dev/null || exit 1   # warm the page cache
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_file -o run --output-format csv -- ./wordcount $F --no-echo --no-list --bench-json gpurun_out/prof_file_bench.json > gpurun_out/prof_file.log 2>&1 || { tail -20 gpurun_out/prof_file.log; exit 1; }
rm -f $F
python3 tools/prof_summary.py gpurun_out/prof_file | head -30
python3 tools/copy_overlap.py gpurun_out/prof_file 4294967296
cat gpurun_out/prof_file_bench.json
