export TMPDIR=/tmp
bash tools/lds_probe.sh > gpurun_out/lds_probe_summary.txt 2>&1 || exit 1
WC_MAP_STAMPS=1 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-oracle > gpurun_out/stamps.out 2> gpurun_out/stamps.err || { tail gpurun_out/stamps.err; exit 1; }
grep -E "hot setup|stamp|phase" gpurun_out/stamps.err | tail -8
cat gpurun_out/lds_probe_summary.txt
