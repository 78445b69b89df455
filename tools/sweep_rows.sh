#!/bin/bash
# Round-3 measurement sweep on one MI355X (every row oracle-validated key for key):
# vocabulary sweep, LONG-word load, 64 GiB config (hot-table reuse A/B), the per-rank
# halves of both 8-GPU configs at full size, merge forced at world 1, kernel trace.
export TMPDIR=/tmp
OUT=gpurun_out/r3s
mkdir -p $OUT
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "FAIL $name"; tail -5 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); st=d['stages']; print('%-28s %8.1f GB/s %8.4f ms/step valid=%s keys=%s dev=%s' % ('$name', d['value'], d['ms_per_step'], d['validated'], d['distinct_words'], st['device_ms']))"
}
if [ $# -gt 0 ]; then  # only the named rows
  for r in "$@"; do
    line=$(grep -E "(^| )run $r " "$0" | grep -v '^ ' | head -1)
    [ -n "$line" ] || { echo "no row $r"; exit 1; }
    eval "$line" || exit 1
  done
  exit 0
fi
run v100k 120 --steps 300 || exit 1
run v500 120 --steps 300 --vocab 500 || exit 1
run v10k 120 --steps 300 --vocab 10000 || exit 1
run v1m 120 --steps 300 --vocab 1000000 || exit 1
run long30_v1m 180 --steps 100 --vocab 1000000 --long-frac 0.3 || exit 1
WC_MERGE_ALWAYS=1 run merge_shuffle 120 --steps 300 --merge shuffle || exit 1
WC_MERGE_ALWAYS=1 run merge_dense 120 --steps 300 --merge dense || exit 1
run c64gb 300 --config 64gb --steps 5 --warmup 1 || exit 1
WC_HOT_RESAMPLE_EVERY=0 run c64gb_sample_every_pass 300 --config 64gb --steps 5 --warmup 1 || exit 1
run c64gb_b 300 --config 64gb --steps 5 --warmup 1 --no-oracle || exit 1
WC_HOT_RESAMPLE_EVERY=0 run c64gb_sample_every_pass_b 300 --config 64gb --steps 5 --warmup 1 --no-oracle || exit 1
WC_MERGE_ALWAYS=1 run c256gb_rank 400 --config 256gb-8gpu --gpus 1 --steps 3 --warmup 1 || exit 1
run c1tb_rank 600 --config 1tb-8gpu-host-staged --gpus 1 --steps 2 --warmup 1 || exit 1
