#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/sort_bench.py || exit 1
WC_MAP_STAMPS=1 WC_LIB=$PWD/cuda_mapreduce_amd/lib/variants/libwc_rstamps.so timeout -k 10 200 python3 bench.py \
  --steps 3 --warmup 1 --no-oracle --vocab 1000000 --long-frac 0.3 > gpurun_out/diag_long.json 2> gpurun_out/diag_long.err
tail -5 gpurun_out/diag_long.err
WC_MAP_STAMPS=1 WC_LIB=$PWD/cuda_mapreduce_amd/lib/variants/libwc_rstamps.so timeout -k 10 200 python3 bench.py \
  --steps 3 --warmup 1 --no-oracle --vocab 1000000 > gpurun_out/diag_v1m.json 2> gpurun_out/diag_v1m.err
tail -5 gpurun_out/diag_v1m.err
