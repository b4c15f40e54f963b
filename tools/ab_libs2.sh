#!/bin/bash
# 32x32 bucket-tree MAR per library variant (base = bn-pp_amd/lib, else
# bn-pp_amd/lib_<name>), per-kernel stats.  usage: tools/ab_libs2.sh base w8 ...
set -o pipefail
R=$PWD
export TMPDIR=/tmp
for v in "$@"; do
  if [ $v = base ]; then L=$R/bn-pp_amd/lib/libbnpp.so; else L=$R/bn-pp_amd/lib_$v/libbnpp.so; fi
  OUT=$R/gpurun_out/abl_$v
  mkdir -p $OUT
  (cd /tmp && BNPP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 > $OUT/log 2>&1) || { tail -5 $OUT/log; exit 1; }
  echo "== $v"; grep -E '"mar"|"check"' $OUT/log | cut -c1-150
  python3 - $OUT/k_kernel_stats.csv <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:6]:
    n = re.sub(r'bnpp::|\(.*', '', r['Name'])
    print("  %-52s %5s calls %8.1f ms  avg %7.3f ms" % (n[:52], r['Calls'], float(r['TotalDurationNs']) / 1e6, float(r['AverageNs']) / 1e6))
PY
done
