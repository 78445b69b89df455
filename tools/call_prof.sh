export TMPDIR=/tmp
WC_MAP_STAMPS=1 timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-oracle 2>&1 | grep -E "image build|phase clock"
for so in cuda_mapreduce_amd/lib/variants/*.so; do
  echo "== $so"; WC_LIB=$PWD/$so WC_MAP_STAMPS=1 timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-oracle 2>&1 | grep -E "image build"
done
