#!/bin/bash
# tools/vbench.sh, then the miss-record count and map / reduce device ms of every run
REPS=${REPS:-3} bash tools/vbench.sh "$@" || exit 1
for f in gpurun_out/vb_*.json; do
  python3 -c "
import json; d=[json.loads(l) for l in open('$f') if l.startswith('{')][-1]
dm=d['stages']['device_ms']; print('%-28s records %d map %.4f reduce %.4f' % ('$f', d['stages']['records'], dm['map'], dm['reduce']))"
done
