#!/bin/bash
# Kernel-time profile of the 1-GPU bench (rocprofv3 --kernel-trace --stats) -> gpurun_out/prof_<tag>
export TMPDIR=/tmp
TAG=${1:-cur}; shift
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 "$@" > gpurun_out/prof_$TAG.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/prof_$TAG | head -24
