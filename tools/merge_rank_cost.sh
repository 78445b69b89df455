#!/bin/bash
# Per-rank merge cost at W virtual ranks: a rocprofv3 kernel
# trace of bench.py --virtual-ranks W for both protocols at 100k and 1M keys per
# rank; tools/merge_rank_cost.py sums each rank's (host thread's) merge-kernel
# device time per step and combines it with the wire bytes the ranks report.
#   tools/merge_rank_cost.sh [W ...]   -> gpurun_out/mrc/*.json + table on stdout
export TMPDIR=/tmp
WS=${*:-1 2 4 8}
mkdir -p gpurun_out/mrc
for vocab in 100000 1000000; do
  for merge in shuffle dense; do
    for w in $WS; do
      tag=w${w}_v${vocab}_$merge
      # W = 1: the protocol forced on (no peer: every kernel uncontended, the per-rank work of an owner)
      WC_MERGE_ALWAYS=1 timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/mrc/$tag -o run --output-format csv \
        -- python3 bench.py --virtual-ranks $w --vocab $vocab --merge $merge --steps 6 --warmup 2 --no-oracle \
        --json-out gpurun_out/mrc/$tag.json > gpurun_out/mrc/$tag.log 2>&1 || { echo "FAILED $tag"; tail -3 gpurun_out/mrc/$tag.log; exit 1; }
      echo "done $tag"
    done
  done
done
python3 tools/merge_rank_cost.py gpurun_out/mrc
