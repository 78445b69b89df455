#!/bin/bash
# Setup-kernel changes: GPU engine/exact tests, interleaved A/B with kernel stats,
# setup-phase stamps of the new build.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_exact.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/setup_tests.log 2>&1 || { tail -20 gpurun_out/setup_tests.log; exit 1; }
tail -1 gpurun_out/setup_tests.log
bash tools/call_ab_ks.sh > gpurun_out/setup_ab.txt 2>&1 || { tail -20 gpurun_out/setup_ab.txt; exit 1; }
grep -E "median|records|wc_hot|wc_map|wc_reduce|wc_fo" gpurun_out/setup_ab.txt | head -40
WC_MAP_STAMPS=1 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-oracle > /dev/null 2> gpurun_out/setup_stamps.err || exit 1
grep -E "hot setup" gpurun_out/setup_stamps.err
