#!/bin/bash
# GPU test suite + 1-GPU bench (tools/gtest.sh [pytest -k expr])
export TMPDIR=/tmp
K=${1:+-k "$1"}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $K > gpurun_out/gtest.log 2>&1
rc=$?
tail -25 gpurun_out/gtest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py > gpurun_out/gtest_bench.json 2> gpurun_out/gtest_bench.err || exit 1
cut -c1-400 gpurun_out/gtest_bench.json
