#!/bin/bash
# Round 5: fp64 split runs with two tiles in flight: identity tests, the fp64
# 32x32 MAR kernel stats.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_bucket_tree.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/mar64 -o mar64 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 1 --reps 2 > $OUT/mar64.log 2>&1 || { tail -5 $OUT/mar64.log; exit 1; }
cd $R
grep -E '"phase": "(mar|check)"' $OUT/mar64.log | cut -c1-200
head -8 $(find $OUT/mar64 -name "*kernel_stats.csv") | cut -c1-160
