#!/bin/bash
# Round 4 (b): slab tile A/B, bench, 32x32 MAR phase split, full GPU suite.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r4b
mkdir -p $OUT
cd $R
timeout -k 10 120 python3 -u $R/tools/slab_ab.py > $OUT/slab_ab.jsonl 2> $OUT/slab_ab.err || exit 1
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
BNPP_TIMING=1 timeout -k 10 200 python3 -u $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 > $OUT/mar.log 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || exit 1
