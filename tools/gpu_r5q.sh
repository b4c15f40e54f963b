#!/bin/bash
# Round 5 probe: fp64 split runs with the bucket arithmetic removed
# (lib_noarith, results wrong, timing only) against the product build.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5q
mkdir -p $OUT
export TMPDIR=/tmp
for v in main noarith; do
  if [ $v = main ]; then unset BNPP_LIB; else export BNPP_LIB=$R/bn-pp_amd/lib_$v/libbnpp.so; fi
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/mar64_$v -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 6 --dtype f64 --check 0 --reps 1 > $OUT/mar64_$v.jsonl 2> $OUT/mar64_$v.err) || { tail -5 $OUT/mar64_$v.err; exit 1; }
  echo "== $v"; head -5 $(find $OUT/mar64_$v -name "*kernel_stats.csv") | cut -c1-160
done
