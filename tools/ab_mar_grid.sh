#!/bin/bash
# 32x32 bucket-tree MAR and per-shape rates at grid-stride (3 workgroups per CU)
# and flat grids, per-kernel stats from rocprofv3.  usage: tools/ab_mar_grid.sh 3 0
set -o pipefail
R=$PWD
export TMPDIR=/tmp
for g in "$@"; do
  OUT=$R/gpurun_out/abg_$g
  mkdir -p $OUT
  (cd /tmp && BNPP_GRID_PER_CU=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 > $OUT/log 2>&1) || { tail -5 $OUT/log; exit 1; }
  echo "== grid_per_cu=$g"; grep '"mar"' $OUT/log | cut -c1-110
  python3 - $OUT/k_kernel_stats.csv <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    n = re.sub(r'bnpp::|\(.*', '', r['Name'])
    print("  %-60s %5s calls %8.1f ms  avg %7.3f ms" % (n[:60], r['Calls'], float(r['TotalDurationNs']) / 1e6, float(r['AverageNs']) / 1e6))
PY
done
