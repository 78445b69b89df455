#!/bin/bash
# tools/kstats.sh for the default build and every variant library (kernel averages side by side):
# tools/kstats_variants.sh [bench args]
for so in cuda_mapreduce_amd/lib/libwc.so cuda_mapreduce_amd/lib/variants/*.so; do
  n=$(basename $so .so)
  WC_LIB=$PWD/$so bash tools/kstats.sh $n "$@" || exit 1
done
