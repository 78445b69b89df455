# The GPU test suite (one process, per-test time limit) + a validated default bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gtest.log 2>&1; rc=$?
tail -5 gpurun_out/gtest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/gtest.log | head -20; exit $rc; }
timeout -k 10 200 python3 bench.py --steps ${STEPS:-200} --warmup 20 > gpurun_out/suite_bench.json 2> gpurun_out/suite_bench.err || { tail -5 gpurun_out/suite_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/suite_bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], 'GB/s', d['ms_per_step'], 'ms valid', d['validated'], d['stages']['device_ms'])"
