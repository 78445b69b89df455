#!/bin/bash
# PMC counters for the map/reduce kernels (own run: --pmc is never combined with tracing).
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  --kernel-include-regex 'wc_map|wc_reduce' -d gpurun_out/pmc1 -o run --output-format csv \
  -- python3 bench.py --steps 2 --warmup 0 > gpurun_out/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES \
  --kernel-include-regex 'wc_map|wc_reduce' -d gpurun_out/pmc2 -o run --output-format csv \
  -- python3 bench.py --steps 2 --warmup 0 > gpurun_out/pmc2.log 2>&1
