#!/bin/bash
# Round 5: where a cold 32x32 MAR's host planning goes (BNPP_TIMING=1), fp32.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5n
mkdir -p $OUT
BNPP_TIMING=1 timeout -k 10 120 python3 -u tools/mar_grid.py --rows 32 --cols 32 --dtype f32 --check 0 --reps 2 > $OUT/mar.jsonl 2> $OUT/mar.err || { tail -20 $OUT/mar.err; exit 1; }
grep "bnpp\]" $OUT/mar.err | head -40
cut -c1-400 $OUT/mar.jsonl
nproc
