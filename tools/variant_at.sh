#!/bin/bash
# Build the engine of git revision REV as a variant library (A/B against the
# working tree in one GPU call): tools/variant_at.sh REV NAME [FLAGS]
# -> cuda_mapreduce_amd/lib/variants/libwc_NAME.so
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2; flags=${3:-}
wt=/tmp/wc_wt_$name
rm -rf $wt && git worktree add -f --detach $wt $rev > /dev/null
(cd $wt && bash tools/variants.sh $name "$flags" > /dev/null)
mkdir -p cuda_mapreduce_amd/lib/variants
cp $wt/cuda_mapreduce_amd/lib/variants/libwc_$name.so cuda_mapreduce_amd/lib/variants/
git worktree remove --force $wt
echo built $name from $rev
