export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
for m in plain shuffle dense; do
  if [ $m = plain ]; then args=""; envs=""; else args="--merge $m"; envs="WC_MERGE_ALWAYS=1"; fi
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tl_$m -o run --output-format csv -- python3 bench.py --steps 10 --warmup 5 --no-oracle $args > gpurun_out/tl_$m.log 2>&1 || { tail -5 gpurun_out/tl_$m.log; exit 1; }
  python3 tools/step_timeline.py gpurun_out/tl_$m > gpurun_out/tl_$m.txt || exit 1
  echo "== $m"; cat gpurun_out/tl_$m.txt
done
