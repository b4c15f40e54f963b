#!/bin/bash
# A/B of the launch grid (BNPP_GRID_PER_CU: 3 = grid-stride over 3 workgroups
# per CU, 0 = flat, one virtual block per workgroup) and the narrow stream tile
# (BNPP_NARROW) on the bench bucket, the per-shape rates and the 32x32 MAR.
set -o pipefail
OUT=gpurun_out/ab_grid
mkdir -p $OUT
for g in 3 0; do
  for n in 0 1; do
    echo "== grid_per_cu=$g narrow=$n" >> $OUT/bench.log
    BNPP_GRID_PER_CU=$g BNPP_NARROW=$n timeout -k 10 120 python3 bench.py --no-cpu --no-mar --steps 20 >> $OUT/bench.log 2>&1 || exit 1
  done
  echo "== grid_per_cu=$g" >> $OUT/shape.log
  BNPP_GRID_PER_CU=$g timeout -k 10 120 python3 tools/shape_bench.py >> $OUT/shape.log 2>&1 || exit 1
done
for g in 3 0; do
  echo "== grid_per_cu=$g" >> $OUT/mar.log
  BNPP_GRID_PER_CU=$g timeout -k 10 200 python3 tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 >> $OUT/mar.log 2>&1 || exit 1
done
