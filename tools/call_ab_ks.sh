# interleaved A/B (vbench_rec) then per-kernel stats of every build
export TMPDIR=/tmp
REPS=${REPS:-3} timeout -k 10 900 bash tools/vbench_rec.sh "$@" || exit 1
bash tools/kstats_ab.sh "$@"
