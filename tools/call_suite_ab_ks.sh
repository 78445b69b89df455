# GPU suite + validated bench, interleaved A/B against the variants, per-kernel stats
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
REPS=${REPS:-3} timeout -k 10 900 bash tools/vbench_rec.sh "$@" || exit 1
bash tools/kstats_ab.sh "$@"
