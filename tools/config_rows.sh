#!/bin/bash
# Every BASELINE config on the shipped build, one call, every row oracle-validated
# (VERDICT r5 item 4): the headline, 64 GiB resident, the per-rank halves of both
# 8-GPU configs at full size (256gb-8gpu with the merge forced on, shuffle and dense;
# 1tb-8gpu-host-staged: 128 GiB over PCIe), then the ./wordcount file path.
# -> gpurun_out/config_rows.txt (+ JSON per row under gpurun_out/cfg/)
export TMPDIR=/tmp
OUT=gpurun_out/cfg
mkdir -p $OUT
R=gpurun_out/config_rows.txt
: > $R
(while sleep 45; do echo "heartbeat $(date +%T)"; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
row() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  echo "running $name" 
  timeout -k 10 $t python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "FAIL $name" | tee -a $R; tail -5 $OUT/$name.err; return 1; }
  python3 - "$OUT/$name.json" "$name" >> $R <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); st = d["stages"]
hp = d.get("host_pool")
print("%-22s %9.1f GB/s %10.4f ms/step  valid=%s  keys=%s  bytes/GPU=%d  chunk=%d  merge=%s  dev=%s%s" % (
    sys.argv[2], d["value"], d["ms_per_step"], d["validated"], d["distinct_words"], d["config"]["bytes_per_gpu"],
    d["config"]["chunk_bytes"], d["config"]["merge"], st["device_ms"],
    ("  pool=%s" % hp) if hp else ""))
PY
  tail -1 $R
}
row v100k 150 --steps 300 || exit 1
row c64gb 300 --config 64gb --steps 5 --warmup 1 || exit 1
WC_MERGE_ALWAYS=1 row c256gb_rank_shuffle 300 --config 256gb-8gpu --gpus 1 --steps 3 --warmup 1 --merge shuffle || exit 1
WC_MERGE_ALWAYS=1 row c256gb_rank_dense 300 --config 256gb-8gpu --gpus 1 --steps 3 --warmup 1 --merge dense || exit 1
row c1tb_rank 600 --config 1tb-8gpu-host-staged --gpus 1 --steps 2 --warmup 1 || exit 1
timeout -k 10 900 bash tools/file_path.sh > $OUT/file_path.log 2>&1 || { echo "FAIL file_path" | tee -a $R; tail -5 $OUT/file_path.log; exit 1; }
cat gpurun_out/file_path.txt >> $R
cat $R
