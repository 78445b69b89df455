#!/bin/bash
# bench.py (no profiler, oracle off) per engine build: default + cuda_mapreduce_amd/lib/variants/*.so
export TMPDIR=/tmp
for so in cuda_mapreduce_amd/lib/libwc.so cuda_mapreduce_amd/lib/variants/*.so; do
  [ -f "$so" ] || continue
  n=$(basename $so .so)
  WC_LIB=$PWD/$so timeout -k 10 150 python3 bench.py --no-oracle "$@" > gpurun_out/vb_$n.json 2> gpurun_out/vb_$n.err
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FAILED $so rc=$rc"; tail -3 gpurun_out/vb_$n.err; exit 1; fi
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/vb_$n.json') if l.startswith('{')][-1]
print('%-14s %8.1f GB/s %7.4f ms' % ('$n', d['value'], d['ms_per_step']))"
done
