#!/bin/bash
# Per-block reduce profile (variant built with -DWC_RED_STAMPS=1 as libwc_rst.so):
# the last job's reduce blocks, slowest first, with their record counts.
# tools/red_blocks.sh TAG [bench args]  -> gpurun_out/rb_TAG.err
export TMPDIR=/tmp
TAG=$1; shift
WC_RED_BLK_ALL=1 WC_STAMPS_PER_JOB=1 WC_MAP_STAMPS=1 WC_LIB=$PWD/cuda_mapreduce_amd/lib/diag/libwc_rst.so timeout -k 10 120 \
  python3 bench.py --steps 2 --warmup 1 --no-oracle "$@" > gpurun_out/rb_$TAG.json 2> gpurun_out/rb_$TAG.err
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -5 gpurun_out/rb_$TAG.err; exit 1; }
echo "== $TAG"; grep -E "reduce|#[0-7]:" gpurun_out/rb_$TAG.err
