#!/bin/bash
# Steady-state A/B for small map changes: the default build and every variant,
# interleaved REPS times, 400 timed steps after 100 warm-up steps (past the
# clock ramp); per run GB/s and the map / reduce device ms of the timed steps.
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=${REPS:-4}
libs="cuda_mapreduce_amd/lib/libwc.so $(ls cuda_mapreduce_amd/lib/variants/*.so 2>/dev/null)"
: > gpurun_out/lab_all.txt
for r in $(seq $REPS); do
  for so in $libs; do
    n=$(basename $so .so)
    WC_LIB=$PWD/$so timeout -k 10 150 python3 bench.py --no-oracle --steps 400 --warmup 100 "$@" > gpurun_out/lab_$n.json 2> gpurun_out/lab_$n.err || { echo "FAILED $so"; tail -3 gpurun_out/lab_$n.err; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/lab_$n.json') if l.startswith('{')][-1]
dm=d['stages']['device_ms']; print('$n', d['value'], dm['map'], dm['reduce'], d['validated'])" | tee -a gpurun_out/lab_all.txt
  done
done
python3 - <<'PY'
import collections, statistics
runs = collections.defaultdict(list)
for line in open("gpurun_out/lab_all.txt"):
    n, v, m, r, ok = line.split()
    runs[n].append((float(v), float(m), float(r)))
for n, v in runs.items():
    print("%-14s median %7.1f GB/s  map %.4f  reduce %.4f ms  runs %s" % (n, statistics.median(x[0] for x in v),
          statistics.median(x[1] for x in v), statistics.median(x[2] for x in v), " ".join("%.1f" % x[0] for x in v)))
PY
