#!/bin/bash
# Kernel traces (default, merge forced at world 1 both protocols, LONG-word load), map/reduce PMC, then the sweep.
export TMPDIR=/tmp
bash tools/kstats.sh cur || exit 1
WC_MERGE_ALWAYS=1 bash tools/kstats.sh shuffle --merge shuffle || exit 1
WC_MERGE_ALWAYS=1 bash tools/kstats.sh dense --merge dense || exit 1
bash tools/kstats.sh long30 --vocab 1000000 --long-frac 0.3 || exit 1
bash tools/pmc_map.sh cur || exit 1
bash tools/r3_sweep.sh
