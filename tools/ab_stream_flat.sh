#!/bin/bash
# (the knob was measured and removed again: profiles/r04_stream_grid_ab.txt)
# Round 4: stream levels on a flat grid (BNPP_STREAM_GRID_PER_CU: workgroups per CU, 0 = flat)
# vs the default grid-stride -- 32x32 MAR wall and the
# stream kernels' summed time from rocprofv3.  usage: tools/ab_stream_flat.sh 3 6 8
set -o pipefail
R=$PWD
export TMPDIR=/tmp
for f in "$@"; do
  OUT=$R/gpurun_out/sflat/f$f
  mkdir -p $OUT
  (cd /tmp && BNPP_STREAM_GRID_PER_CU=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 > $OUT/log 2>&1) || { tail -5 $OUT/log; exit 1; }
  echo "== stream_grid_per_cu=$f"; grep '"mar"' $OUT/log | cut -c1-110
  python3 - $OUT/k_kernel_stats.csv <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows) / 1e6
st = [r for r in rows if 'stream_level' in r['Name']]
print("  all kernels %.1f ms, stream_level %.1f ms" % (tot, sum(float(r['TotalDurationNs']) for r in st) / 1e6))
for r in sorted(st, key=lambda r: -float(r['TotalDurationNs']))[:6]:
    n = re.sub(r'bnpp::|\(.*', '', r['Name'])
    print("  %-60s %5s calls %8.1f ms  max %7.3f ms" % (n[:60], r['Calls'], float(r['TotalDurationNs']) / 1e6, float(r['MaxNs']) / 1e6))
PY
done
