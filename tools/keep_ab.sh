#!/bin/bash
# 32x32 MAR wall-clock per BNPP_KEEP_LOG2 value
set -o pipefail
for k in "$@"; do
  echo "== keep $k"
  BNPP_KEEP_LOG2=$k timeout -k 10 200 python3 tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 2>&1 | grep -E '"mar"|"check"|"plan"' | cut -c1-220 || exit 1
done
