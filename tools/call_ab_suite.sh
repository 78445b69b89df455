# GPU suite + validated bench of the working tree, then an interleaved A/B against the variants.
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
REPS=${REPS:-3} timeout -k 10 900 bash tools/vbench_rec.sh "$@"
