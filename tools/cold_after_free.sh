#!/bin/bash
# Is a cold MAR call slow because the previous process just freed ~250 GB of
# HBM (the driver clearing returned pages)?  A: back-to-back processes;
# B: the same with 15 s between them.  (run on the GPU box from the repo root)
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/caf
mkdir -p $OUT
M="python3 -u $R/tools/mar_grid.py --rows 32 --cols 32 --check 0"
timeout -k 10 120 $M --reps 1 > $OUT/a0.log 2>&1 || exit 1
timeout -k 10 120 $M --reps 2 > $OUT/a1.log 2>&1 || exit 1
sleep 15
timeout -k 10 120 $M --reps 2 > $OUT/b1.log 2>&1 || exit 1
grep -h '"phase": "mar"' $OUT/a0.log $OUT/a1.log $OUT/b1.log
