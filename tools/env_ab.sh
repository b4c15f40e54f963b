#!/bin/bash
# 32x32 bucket-tree MAR wall-clock under each environment setting given as an
# argument ("-" = none), e.g.  tools/env_ab.sh - BNPP_NO_REDUCE_MANY=1
set -o pipefail
for e in "$@"; do
  echo "== $e"
  if [ "$e" = "-" ]; then
    timeout -k 10 200 python3 tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 2>&1 | grep -E '"mar"|"check"|"plan"' | cut -c1-200 || exit 1
  else
    env "$e" timeout -k 10 200 python3 tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 2>&1 | grep -E '"mar"|"check"|"plan"' | cut -c1-200 || exit 1
  fi
done
