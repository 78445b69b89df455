# (1) the setup kernels' phase clock; (2) the round-4 t17 test once under a kernel trace
export TMPDIR=/tmp
WC_MAP_STAMPS=1 timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-oracle 2>&1 | grep -E "hot setup|phase clock"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/t17 -o run --output-format csv \
  -- python3 -m pytest tests/test_gpu_exact.py::test_reset_ignores_stale_slices -x -q > gpurun_out/t17.log 2>&1
echo "t17 rc=$?"; tail -3 gpurun_out/t17.log
