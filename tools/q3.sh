#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q3_tests.log 2>&1 || { tail -30 gpurun_out/q3_tests.log; exit 1; }
tail -1 gpurun_out/q3_tests.log
bash tools/vrun.sh
