#!/bin/bash
# PMC counters of wc_map_tokenize, current kernel vs WC_MAP_V4=1 (each pass its own run, no tracing).
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH"
for v in 0 1; do
  for p in 1 2; do
    eval C=\$P$p
    WC_MAP_V4=$v timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'wc_map' -d gpurun_out/pmc_v${v}_$p -o run --output-format csv \
      -- python3 bench.py --steps 1 --warmup 0 > gpurun_out/pmc_v${v}_$p.log 2>&1 || exit 1
  done
done
echo done
