#!/bin/bash
# GPU suite with every device allocation poisoned (WC_POISON=1: 0xA5 fill at
# hipMalloc; =2: also every DeviceArena region at reuse) — a kernel or host path
# that depends on fresh memory reading as zero fails deterministically here.
# tools/poison_suite.sh [level]   -> gpurun_out/poison_<level>.log
export TMPDIR=/tmp
L=${1:-1}
WC_POISON=$L timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/poison_$L.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/poison_$L.log | tail -3
exit $rc
