#!/bin/bash
# Bench each built variant (and the default build) on the same box: tools/vrun.sh [bench args]
# (ablation variants fail validation by design: their numbers are timings only)
export TMPDIR=/tmp
for so in cuda_mapreduce_amd/lib/libwc.so cuda_mapreduce_amd/lib/variants/*.so cuda_mapreduce_amd/lib/libwc.so; do
  [ -f "$so" ] || continue
  WC_LIB=$PWD/$so timeout -k 10 120 python bench.py "$@" > gpurun_out/vrun.json 2>gpurun_out/vrun.err
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FAILED $so rc=$rc"; tail -3 gpurun_out/vrun.err; exit 1; fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/vrun.json').read()); st=d['stages']; print('%-28s %8.1f GB/s  %.3f ms  mr %.3f fin %.3f  records %.1fM reruns %d splits %d valid %s' % (sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], st['map_reduce_ms'], st['finalize_ms'], st['records']/1e6, st['map_reruns'], st['table_splits'], d.get('validated')))" $so
done
