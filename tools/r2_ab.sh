#!/bin/bash
# A/B of built variants on one box: GPU tests (default build), kernel times, benches
bash tools/quick.sh && bash tools/stamps.sh && bash tools/vprof.sh && bash tools/vrun.sh
