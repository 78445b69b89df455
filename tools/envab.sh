#!/bin/bash
# Interleaved A/B of one environment switch on bench.py (every run oracle-validated):
#   tools/envab.sh VAR "VAL_A VAL_B" REPS [bench args]   -> medians per value
export TMPDIR=/tmp
VAR=$1; VALS=$2; REPS=$3; shift 3
: > gpurun_out/envab.txt
for r in $(seq $REPS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 150 python3 bench.py --steps 100 --warmup 10 "$@" > gpurun_out/envab_$v.json 2> gpurun_out/envab_$v.err
    rc=$?
    [ $rc -eq 0 ] || { echo "FAILED $VAR=$v rc=$rc"; tail -3 gpurun_out/envab_$v.err; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/envab_$v.json') if l.startswith('{')][-1]
st=d['stages']['device_ms']
print('$v', d['value'], d['validated'], st['map'], st['reduce'], st['finalize'])" >> gpurun_out/envab.txt
  done
done
python3 - "$VAR" "$*" <<'PY'
import collections, statistics, sys
runs = collections.defaultdict(list)
for line in open("gpurun_out/envab.txt"):
    v, g, ok, m, r, f = line.split()
    runs[v].append((float(g), ok, float(m), float(r), float(f)))
for v, x in runs.items():
    print("%s=%-4s median %7.1f GB/s  valid %s  map %.3f reduce %.3f fin %.3f  runs %s  %s" % (
        sys.argv[1], v, statistics.median(a[0] for a in x), all(a[1] == "True" for a in x),
        statistics.median(a[2] for a in x), statistics.median(a[3] for a in x), statistics.median(a[4] for a in x),
        " ".join("%.1f" % a[0] for a in x), sys.argv[2]))
PY
