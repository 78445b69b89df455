#!/bin/bash
# End-to-end bench.py GB/s of the default build and every variant in
# cuda_mapreduce_amd/lib/variants, interleaved (A B C A B C ...) REPS times,
# 50 timed steps each; prints every run and the median per build.
# tools/vbench.sh [bench args]   (REPS=3 by default)
export TMPDIR=/tmp
REPS=${REPS:-3}
libs="cuda_mapreduce_amd/lib/libwc.so $(ls cuda_mapreduce_amd/lib/variants/*.so 2>/dev/null)"
: > gpurun_out/vb_all.txt
for r in $(seq $REPS); do
  for so in $libs; do
    n=$(basename $so .so)
    WC_LIB=$PWD/$so timeout -k 10 150 python3 bench.py --no-oracle --steps 50 --warmup 10 "$@" > gpurun_out/vb_$n.json 2> gpurun_out/vb_$n.err
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FAILED $so rc=$rc"; tail -3 gpurun_out/vb_$n.err; exit 1; fi
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/vb_$n.json') if l.startswith('{')][-1]
print('$n', d['value'])" >> gpurun_out/vb_all.txt
  done
done
python3 - "$*" <<'PY'
import collections, statistics, sys
runs = collections.defaultdict(list)
for line in open("gpurun_out/vb_all.txt"):
    n, v = line.split()
    runs[n].append(float(v))
for n, v in runs.items():
    print("%-14s median %7.1f GB/s  runs %s  %s" % (n, statistics.median(v), " ".join("%.1f" % x for x in v), sys.argv[1]))
PY
