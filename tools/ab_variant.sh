#!/bin/bash
# A/B of one variant (cuda_mapreduce_amd/lib/variants/libwc_NAME.so) against the default build:
# the map/reduce exactness tests on the variant, then the interleaved bench (tools/vbench.sh).
# tools/ab_variant.sh NAME [bench args]
export TMPDIR=/tmp
NAME=$1; shift
WC_LIB=$PWD/cuda_mapreduce_amd/lib/variants/libwc_$NAME.so timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py \
  tests/test_gpu_exact.py tests/test_gpu_order.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_$NAME.log 2>&1
rc=$?; tail -3 gpurun_out/ab_$NAME.log; [ $rc -eq 0 ] || exit $rc
REPS=${REPS:-4} bash tools/vbench.sh "$@"
