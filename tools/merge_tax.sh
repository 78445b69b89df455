#!/bin/bash
# Merged-finalize tax at world size 1: bench.py plain vs
# the RCCL merge protocol forced on (WC_MERGE_ALWAYS=1) for shuffle and dense,
# interleaved REPS times (the planned merge runs from the second job on).
#   tools/merge_tax.sh [bench args]   -> gpurun_out/merge_tax.txt
export TMPDIR=/tmp
REPS=${REPS:-2}
OUT=gpurun_out/merge_tax.txt
: > $OUT
for r in $(seq $REPS); do
  for m in plain shuffle dense; do
    if [ $m = plain ]; then
      timeout -k 10 200 python3 bench.py --no-oracle --steps 200 --warmup 10 "$@" > /tmp/mt.json 2> /tmp/mt.err
    else
      WC_MERGE_ALWAYS=1 timeout -k 10 200 python3 bench.py --no-oracle --steps 200 --warmup 10 --merge $m "$@" \
        > /tmp/mt.json 2> /tmp/mt.err
    fi
    rc=$?
    if [ $rc -ne 0 ]; then echo "merge_tax $m rc=$rc"; tail -3 /tmp/mt.err; exit 1; fi
    python3 -c "
import json; d=[json.loads(l) for l in open('/tmp/mt.json') if l.startswith('{')][-1]; s=d['stages']
print('$m', d['ms_per_step'], d['value'], s['device_ms']['merge'], s.get('merges_planned', 0), s.get('merge_redos', 0))" >> $OUT
  done
done
python3 - <<'PY'
import collections, statistics
rows = collections.defaultdict(list)
for line in open("gpurun_out/merge_tax.txt"):
    m, ms, gbs, mg, pl, rd = line.split()
    rows[m].append((float(ms), float(gbs), float(mg), int(pl), int(rd)))
base = statistics.median(r[0] for r in rows["plain"])
for m, v in rows.items():
    ms = statistics.median(r[0] for r in v)
    print("%-8s ms/step %.4f  tax %.3fx  GB/s %.1f  merge stage %.4f ms  planned merges %d redos %d" % (
        m, ms, ms / base, statistics.median(r[1] for r in v), statistics.median(r[2] for r in v), v[-1][3], v[-1][4]))
PY
