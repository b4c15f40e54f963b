#!/bin/bash
# 32x32 bucket-tree MAR with the split chain forms (runs of up to 8 buckets,
# chainsplit.cuh) and without (BNPP_NO_SPLIT=1: one-thread runs of <= 6), kernel
# stats from rocprofv3.  usage: tools/ab_split.sh
set -o pipefail
R=$PWD
export TMPDIR=/tmp
for ns in ${SPLIT_SET:-0 1}; do
  OUT=$R/gpurun_out/split_$ns
  mkdir -p $OUT
  (cd /tmp && BNPP_NO_SPLIT=$ns timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 > $OUT/log 2>&1) || { tail -5 $OUT/log; exit 1; }
  echo "== no_split=$ns"; grep -E '"mar"|"check"' $OUT/log | cut -c1-160
  python3 - $OUT/k_kernel_stats.csv <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:9]:
    n = re.sub(r'bnpp::|\(.*', '', r['Name'])
    print("  %-52s %5s calls %8.1f ms  avg %7.3f ms" % (n[:52], r['Calls'], float(r['TotalDurationNs']) / 1e6, float(r['AverageNs']) / 1e6))
PY
done
