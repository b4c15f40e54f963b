#!/bin/bash
# A/B library variants (tools/build_variant.sh) on tools/shape_bench.py and,
# with AB_MAR=1, the 32x32 bucket-tree MAR.   usage: tools/ab_shapes.sh base v1 v2 ...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  if [ $v = base ]; then L=$PWD/bn-pp_amd/lib/libbnpp.so; else L=$PWD/bn-pp_amd/lib_$v/libbnpp.so; fi
  echo "== $v"
  BNPP_LIB=$L timeout -k 10 300 python tools/shape_bench.py --n 29 > gpurun_out/abs_$v.jsonl 2>&1 || { tail -5 gpurun_out/abs_$v.jsonl; exit 1; }
  grep shape gpurun_out/abs_$v.jsonl
  if [ -n "$AB_MAR" ]; then
    BNPP_LIB=$L timeout -k 10 600 python tools/mar_grid.py --rows 32 --cols 32 --check 0 > gpurun_out/abm_$v.jsonl 2>&1 || { tail -5 gpurun_out/abm_$v.jsonl; exit 1; }
    grep '"mar"' gpurun_out/abm_$v.jsonl | cut -c1-160
  fi
done
