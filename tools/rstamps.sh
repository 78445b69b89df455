#!/bin/bash
# Reduce diagnostic counters (variant built with -DWC_RED_STAMPS=1 as libwc_rst.so): tools/rstamps.sh [bench args]
export TMPDIR=/tmp
WC_MAP_STAMPS=1 WC_LIB=$PWD/cuda_mapreduce_amd/lib/diag/libwc_rst.so timeout -k 10 120 python3 bench.py --steps 1 --warmup 0 --no-oracle "$@" \
  > gpurun_out/rst.json 2> gpurun_out/rst.err; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -5 gpurun_out/rst.err; exit 1; }
grep "reduce counters\|map phase" gpurun_out/rst.err
