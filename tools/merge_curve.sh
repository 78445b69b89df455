#!/bin/bash
# Merge-stage cost at W virtual ranks on one GPU (bench.py --virtual-ranks W:
# W engines in threads, the stream-ordered loopback communicator, 1 GiB shard
# each, oracle-validated): W = 2 4 8, 100k and 1M words, both protocols.
#   tools/merge_curve.sh [W ...]      -> gpurun_out/merge_curve.jsonl
export TMPDIR=/tmp
WS=${*:-2 4 8}
mkdir -p gpurun_out
: > gpurun_out/merge_curve.jsonl
for vocab in 100000 1000000; do
  for merge in shuffle dense; do
    for w in $WS; do
      timeout -k 10 300 python3 bench.py --virtual-ranks $w --vocab $vocab --merge $merge --steps 10 --warmup 2 \
        >> gpurun_out/merge_curve.jsonl 2> gpurun_out/merge_curve_$w.err
      rc=$?
      if [ $rc -ne 0 ]; then echo "virtual ranks W=$w vocab=$vocab $merge: rc=$rc"; tail -3 gpurun_out/merge_curve_$w.err; exit 1; fi
      tail -1 gpurun_out/merge_curve.jsonl | python3 -c "
import json, sys; d = json.loads(sys.stdin.read())
print('W=%d vocab=%s %-7s validated=%s ms/step=%.3f merge_ms(max)=%.3f stages0=%s' % (d['virtual_ranks'], d['config']['vocab'],
      d['config']['merge'], d['validated'], d['ms_per_step'], max(d['merge_ms']), d['stage_ms_rank0']))"
    done
  done
done
