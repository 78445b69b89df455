export TMPDIR=/tmp
WC_MAP_STAMPS=1 timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-oracle 2>&1 | grep -E "hot setup"
bash tools/call_ab_ks.sh "$@"
