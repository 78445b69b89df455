#!/bin/bash
# Merged step (protocol forced on at world 1, WC_MERGE_ALWAYS=1) of the default
# build against every variant in cuda_mapreduce_amd/lib/variants, interleaved
# REPS times: ms / step and the merge stage per build.
#   tools/merge_ab.sh shuffle|dense [bench args]   -> gpurun_out/merge_ab.txt
export TMPDIR=/tmp
REPS=${REPS:-3}
M=$1; shift
libs="cuda_mapreduce_amd/lib/libwc.so $(ls cuda_mapreduce_amd/lib/variants/*.so 2>/dev/null)"
: > gpurun_out/merge_ab.txt
for r in $(seq $REPS); do
  for so in $libs; do
    n=$(basename $so .so)
    WC_LIB=$PWD/$so WC_MERGE_ALWAYS=1 timeout -k 10 200 python3 bench.py --no-oracle --steps 200 --warmup 10 \
      --merge $M "$@" > /tmp/ma.json 2> /tmp/ma.err || { echo "FAILED $n"; tail -3 /tmp/ma.err; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('/tmp/ma.json') if l.startswith('{')][-1]
print('$n', d['ms_per_step'], d['stages']['device_ms']['merge'])" >> gpurun_out/merge_ab.txt
  done
done
python3 - "$M $*" <<'PY'
import collections, statistics, sys
runs = collections.defaultdict(list)
for line in open("gpurun_out/merge_ab.txt"):
    n, ms, mg = line.split()
    runs[n].append((float(ms), float(mg)))
for n, v in runs.items():
    print("%-14s ms/step %.4f  merge stage %.4f ms  runs %s  %s" % (
        n, statistics.median(a[0] for a in v), statistics.median(a[1] for a in v),
        " ".join("%.4f" % a[0] for a in v), sys.argv[1]))
PY
