#!/bin/bash
# Round 5: fp64 split runs of 8 buckets (aliased LDS): bucket-tree and parity
# tests, then the fp64 32x32 MAR with its kernel trace.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_bucket_tree.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/mar64 -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 3 --reps 2 > $OUT/mar64.jsonl 2> $OUT/mar64.err) || { tail -5 $OUT/mar64.err; exit 1; }
grep -h '"mar"\|check' $OUT/mar64.jsonl | cut -c1-200
head -12 $(find $OUT/mar64 -name "*kernel_stats.csv") | cut -c1-160
