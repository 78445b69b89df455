#!/bin/bash
# vprof over the default + variant builds (rst excluded: diagnostic), then the rst counters
export TMPDIR=/tmp
mkdir -p /tmp/rst && mv cuda_mapreduce_amd/lib/variants/libwc_rst.so /tmp/rst/ 2>/dev/null
bash tools/vprof.sh --no-oracle "$@"; rc=$?
mv /tmp/rst/libwc_rst.so cuda_mapreduce_amd/lib/variants/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
bash tools/rstamps.sh --steps 3 "$@"
