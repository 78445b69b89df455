#!/bin/bash
# Full GPU test suite, then the A/B of tools/r3_ab.sh's bench part and a kernel trace
# (tools/r3_full.sh [bench args])
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3_full_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_full_tests.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/r3_full_tests.log | head -20; exit $rc; }
REPS=${REPS:-4} bash tools/vbench.sh "$@" && bash tools/kstats.sh new "$@"
