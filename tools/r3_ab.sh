#!/bin/bash
# A/B: working-tree build vs the variants in cuda_mapreduce_amd/lib/variants (interleaved),
# after the GPU tests that exercise the map, reduce and finalize (tools/r3_ab.sh [bench args])
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_exact.py tests/test_gpu_props.py \
  tests/test_gpu_order.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_ab_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=${REPS:-4} bash tools/vbench.sh "$@"
