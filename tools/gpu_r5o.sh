#!/bin/bash
# Round 5: fp64 one-run split kernels with the row image on the exchange table
# (two workgroups per CU): bucket-tree tests, then the fp64 32x32 MAR with the
# product build and without the aliasing (lib_noalias), kernel traces.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_bucket_tree.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in main noalias; do
  if [ $v = main ]; then unset BNPP_LIB; else export BNPP_LIB=$R/bn-pp_amd/lib_$v/libbnpp.so; fi
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/mar64_$v -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 1 --reps 2 > $OUT/mar64_$v.jsonl 2> $OUT/mar64_$v.err) || { tail -5 $OUT/mar64_$v.err; exit 1; }
  echo "== $v"; grep -h '"mar"\|check' $OUT/mar64_$v.jsonl | cut -c1-200
  head -5 $(find $OUT/mar64_$v -name "*kernel_stats.csv") | cut -c1-160
done
