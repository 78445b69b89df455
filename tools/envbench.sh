#!/bin/bash
# End-to-end bench.py GB/s under different environment settings, interleaved
# REPS times (50 timed steps each); prints every run and the median per setting.
# tools/envbench.sh "WC_SORT_COOP=1" "WC_SORT_COOP=0" [-- bench args]
export TMPDIR=/tmp
REPS=${REPS:-3}
envs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
[ "$1" = "--" ] && shift
: > gpurun_out/eb_all.txt
for r in $(seq $REPS); do
  for i in "${!envs[@]}"; do
    e=${envs[$i]}
    env $e timeout -k 10 150 python3 bench.py --no-oracle --steps 50 --warmup 10 "$@" > gpurun_out/eb_$i.json 2> gpurun_out/eb_$i.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "FAILED [$e] rc=$rc"; tail -3 gpurun_out/eb_$i.err; exit 1; fi
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/eb_$i.json') if l.startswith('{')][-1]
dm=d['stages']['device_ms']; print('$i', d['value'], dm['map'], dm['reduce'])" >> gpurun_out/eb_all.txt
  done
done
python3 - "$*" "${envs[@]}" <<'PY'
import collections, statistics, sys
names = sys.argv[2:]
runs = collections.defaultdict(list)
for line in open("gpurun_out/eb_all.txt"):
    i, v, m, r = line.split()
    runs[int(i)].append((float(v), float(m), float(r)))
for i, v in sorted(runs.items()):
    print("%-28s median %7.1f GB/s  map %.4f reduce %.4f ms  runs %s  %s" % (
        names[i], statistics.median(x[0] for x in v), statistics.median(x[1] for x in v),
        statistics.median(x[2] for x in v), " ".join("%.1f" % x[0] for x in v), sys.argv[1]))
PY
