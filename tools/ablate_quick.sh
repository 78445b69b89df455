export TMPDIR=/tmp
for m in ${MODES:-0 7 5 1 0}; do
  WC_ABLATE_MAP=$m timeout -k 10 120 python bench.py --steps 5 --warmup 1 > gpurun_out/abl_$m.json 2>/dev/null
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/abl_$m.json').read()); st=d['stages']; print('ablate $m', d['ms_per_step'], 'mr', st['map_reduce_ms'], 'records', st['records'])"
done
