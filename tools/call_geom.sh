set -o pipefail
REPS=2 timeout -k 10 600 bash tools/vbench_rec.sh > gpurun_out/geom_ab.txt 2>&1; echo vb_rc=$?
cat gpurun_out/geom_ab.txt
WC_LIB=$PWD/cuda_mapreduce_amd/lib/variants/libwc_t512s6k.so timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 > gpurun_out/t512s6k_valid.json 2>&1; echo valid_rc=$?
python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/t512s6k_valid.json') if l.startswith('{')][-1]; print('t512s6k validated', d['validated'], d['value'])"
bash tools/rccl_one_gpu.sh --steps 5 --warmup 1 > gpurun_out/rccl1g.txt 2>&1; echo rccl_rc=$?
tail -30 gpurun_out/rccl1g.txt
