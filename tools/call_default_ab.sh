#!/bin/bash
# bench.py defaults (1000 timed steps, oracle-validated) of the default build
# and every variant, interleaved REPS times
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=${REPS:-3}
libs="cuda_mapreduce_amd/lib/libwc.so $(ls cuda_mapreduce_amd/lib/variants/*.so 2>/dev/null)"
: > gpurun_out/dab_all.txt
for r in $(seq $REPS); do
  for so in $libs; do
    n=$(basename $so .so)
    WC_LIB=$PWD/$so timeout -k 10 200 python3 bench.py > gpurun_out/dab_$n.json 2> gpurun_out/dab_$n.err || { echo "FAILED $so"; tail -3 gpurun_out/dab_$n.err; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/dab_$n.json') if l.startswith('{')][-1]
dm=d['stages']['device_ms']; print('$n', d['value'], dm['map'], dm['reduce'], d['validated'])" | tee -a gpurun_out/dab_all.txt
  done
done
