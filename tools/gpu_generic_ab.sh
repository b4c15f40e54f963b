#!/bin/bash
# A/B of the generic kernels built with and without SimplifyCFG's store
# sinking (tools/generic_ab.py under rocprofv3 --kernel-trace --stats).
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/generic_ab
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for v in base split base2 split2; do
  L=${v%2}
  BNPP_LIB=$R/build_ab/libbnpp_$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o k --output-format csv -- python3 $R/tools/generic_ab.py > $OUT/$v.jsonl 2> $OUT/$v.err || { tail -5 $OUT/$v.err; exit 1; }
done
