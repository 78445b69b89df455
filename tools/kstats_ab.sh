# tools/kstats.sh for the working tree and every variant library (per-kernel averages, one call)
export TMPDIR=/tmp
bash tools/kstats.sh cur "$@" || exit 1
for so in cuda_mapreduce_amd/lib/variants/*.so; do
  n=$(basename $so .so)
  WC_LIB=$PWD/$so bash tools/kstats.sh $n "$@" || exit 1
done
