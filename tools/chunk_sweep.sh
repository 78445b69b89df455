export TMPDIR=/tmp
for r in 1 2; do
for c in 1 0.5 0.25; do
  timeout -k 10 120 python3 bench.py --no-oracle --steps 50 --warmup 10 --chunk-gb $c > gpurun_out/ch.json 2>/dev/null || exit 1
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/ch.json') if l.startswith('{')][-1]
print('chunk $c', d['value'], d['stages']['device_ms'])"
done; done
