set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/g1_tests.log 2>&1
timeout -k 10 180 python bench.py > gpurun_out/g1_bench.json 2> gpurun_out/g1_bench.err
cat gpurun_out/g1_bench.json
