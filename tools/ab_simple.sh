#!/bin/bash
# Per-target MAR (12x32 and 10x10, fp64) with small buckets merged into one
# generic launch per level up to BNPP_SIMPLE_MAX output entries.  (GPU box)
R=$PWD
for sm in 0 4096 65536 262144; do
  echo "== simple_max=$sm"
  BNPP_SIMPLE_MAX=$sm BNPP_TIMING=1 timeout -k 10 120 python3 -u tools/pertarget_timing.py > $R/gpurun_out/sm_$sm.log 2>&1 || exit 1
  grep -E "^mar|launches|marginals:" $R/gpurun_out/sm_$sm.log | tail -3
done
