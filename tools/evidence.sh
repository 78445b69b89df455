#!/bin/bash
# Evidence bundle for profiles/: kernel trace stats, phase clock, config sweep (1 GPU).
export TMPDIR=/tmp
bash tools/prof.sh r1 > gpurun_out/evidence_prof.txt 2>&1 || { cat gpurun_out/evidence_prof.txt; exit 1; }
WC_MAP_STAMPS=1 timeout -k 10 120 python bench.py --steps 3 --warmup 1 2>&1 | grep "phase clock" > gpurun_out/evidence_phase.txt || exit 1
WC_MAP_STAMPS=1 timeout -k 10 120 python bench.py --steps 3 --warmup 1 --vocab 500 2>&1 | grep "phase clock" >> gpurun_out/evidence_phase.txt || exit 1
bash tools/sweep.sh > gpurun_out/evidence_sweep.txt 2>&1 || { cat gpurun_out/evidence_sweep.txt; exit 1; }
cat gpurun_out/evidence_prof.txt gpurun_out/evidence_phase.txt gpurun_out/evidence_sweep.txt | cut -c1-200
