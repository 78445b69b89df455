#!/bin/bash
# End-of-session validation: full GPU suite, smoke(), driver-style default bench, sweep rows
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1
rc=$?; tail -3 gpurun_out/final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -5 gpurun_out/final_bench.err; exit 1; }
tail -1 gpurun_out/final_bench.json | cut -c1-400
bash tools/r3_sweep.sh v100k v10k v1m long30_v1m merge_shuffle merge_dense c64gb
