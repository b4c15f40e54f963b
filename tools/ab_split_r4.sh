#!/bin/bash
# Round 4: split-run variants on the 32x32 MAR (kernel stats per variant
# library via BNPP_LIB) and the bare replica (tools/splitbw.hip) on the same
# box.  usage (GPU box, repo root): tools/ab_split_r4.sh base bwd2
set -o pipefail
R=$PWD
export TMPDIR=/tmp
OUTR=$R/gpurun_out/ab4
mkdir -p $OUTR
timeout -k 10 120 $R/build/splitbw > $OUTR/splitbw.jsonl 2>&1 || exit 1
for v in "$@"; do
  OUT=$OUTR/$v
  mkdir -p $OUT
  LIB=$R/bn-pp_amd/lib/libbnpp.so
  [ "$v" != base ] && LIB=$R/bn-pp_amd/lib_$v/libbnpp.so
  (cd /tmp && BNPP_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 > $OUT/log 2>&1) || { tail -5 $OUT/log; exit 1; }
  echo "== $v"; grep -E '"mar"|"check"' $OUT/log | cut -c1-200
  python3 - $OUT/k_kernel_stats.csv <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:4]:
    n = re.sub(r'bnpp::|\(.*', '', r['Name'])
    print("  %-52s %5s calls %8.1f ms  avg %7.3f ms" % (n[:52], r['Calls'], float(r['TotalDurationNs']) / 1e6, float(r['AverageNs']) / 1e6))
PY
done
