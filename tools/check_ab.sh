#!/bin/bash
# One gpurun call: GPU test suite, a validated bench.py run, then the A/B of
# the working-tree build against every variant in cuda_mapreduce_amd/lib/variants
# (end-to-end GB/s, interleaved) and their kernel times.
#   tools/check_ab.sh [TAG]      (REPS=3 interleaved bench runs per build)
export TMPDIR=/tmp
TAG=${1:-ab}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_gtest.log 2>&1
rc=$?
tail -4 gpurun_out/${TAG}_gtest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests rc=$rc: stopping"; exit 1; fi
timeout -k 10 300 python bench.py --steps 200 --warmup 10 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?
cut -c1-400 gpurun_out/${TAG}_bench.json; tail -3 gpurun_out/${TAG}_bench.err
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "bench rc=$rc: stopping"; exit 1; fi
REPS=${REPS:-3} bash tools/vbench.sh || exit 1
bash tools/vprof.sh
