#!/bin/bash
# Round-4 cold-mapping probe (run on the GPU box from the repo root).
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r4probe
mkdir -p $OUT
timeout -k 10 200 $R/tools/map_probe 240 > $OUT/map_probe.log 2>&1 || exit 1
BNPP_TIMING=1 timeout -k 10 200 python3 -u $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 > $OUT/mar.log 2>&1 || exit 1
