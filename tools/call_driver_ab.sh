#!/bin/bash
# the driver's bench shape (20 timed steps after 5 warm-up) of the default
# build and every variant, one process each, interleaved REPS times
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=${REPS:-4}
libs="cuda_mapreduce_amd/lib/libwc.so $(ls cuda_mapreduce_amd/lib/variants/*.so 2>/dev/null)"
: > gpurun_out/drv_all.txt
for r in $(seq $REPS); do
  for so in $libs; do
    n=$(basename $so .so)
    WC_LIB=$PWD/$so timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv_$n.json 2> gpurun_out/drv_$n.err || { echo "FAILED $so"; tail -3 gpurun_out/drv_$n.err; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/drv_$n.json') if l.startswith('{')][-1]
dm=d['stages']['device_ms']; print('$n', d['value'], dm['map'], dm['reduce'], d['validated'])" | tee -a gpurun_out/drv_all.txt
  done
done
python3 - <<'PY'
import collections, statistics
runs = collections.defaultdict(list)
for line in open("gpurun_out/drv_all.txt"):
    n, v, m, r, ok = line.split()
    runs[n].append((float(v), float(m)))
for n, v in runs.items():
    print("%-14s median %7.1f GB/s  map %.4f ms  runs %s" % (n, statistics.median(x[0] for x in v),
          statistics.median(x[1] for x in v), " ".join("%.1f" % x[0] for x in v)))
PY
