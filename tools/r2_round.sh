#!/bin/bash
# One gpurun call: GPU tests + 1-GPU bench, torchrun launcher path, kernel profile.
mkdir -p gpurun_out
bash tools/gtest.sh && bash tools/dist_smoke.sh && bash tools/prof.sh "${1:-r2}"
