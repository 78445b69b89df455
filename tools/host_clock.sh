# Host milestones per job (WC_HOST_CLOCK=1, printed at teardown) for the plain
# and the forced-merge steps: where the GPU idle gap between jobs goes.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
for m in plain shuffle dense; do
  if [ $m = plain ]; then args=""; envs=""; else args="--merge $m"; envs="WC_MERGE_ALWAYS=1"; fi
  env $envs WC_HOST_CLOCK=1 timeout -k 10 200 python3 bench.py --steps 100 --warmup 10 --no-oracle $args \
    > gpurun_out/hc_$m.json 2> gpurun_out/hc_$m.err || { tail -5 gpurun_out/hc_$m.err; exit 1; }
  echo "== $m $(python3 -c "import json;d=json.loads(open('gpurun_out/hc_$m.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
  grep "host clock" gpurun_out/hc_$m.err || true
done
