#!/bin/bash
# Round 4: slab form with outer dims vs the stream kernel on the 32x32 MAR's
# first-column buckets -- wall and per-kernel totals from rocprofv3 under each
# environment setting ("-" = none).  usage: tools/ab_slab_outer.sh - BNPP_NO_SLAB_OUTER=1
set -o pipefail
R=$PWD
export TMPDIR=/tmp
for e in "$@"; do
  tag=$(echo "$e" | tr '= ' '_+')
  OUT=$R/gpurun_out/slabo/$tag
  mkdir -p $OUT
  if [ "$e" = "-" ]; then e="BNPP_AB_NONE=1"; fi
  (cd /tmp && for kv in $e; do export $kv; done && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 > $OUT/log 2>&1) || { tail -5 $OUT/log; exit 1; }
  echo "== $e"; grep -E '"mar"|"check"' $OUT/log | cut -c1-160
  python3 - $OUT/k_kernel_stats.csv <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows) / 1e6
def s(key): return sum(float(r['TotalDurationNs']) for r in rows if key in r['Name']) / 1e6
print("  all kernels %.1f ms, stream_level %.1f ms, slab_level %.1f ms" % (tot, s('stream_level'), s('slab_level')))
for r in sorted([r for r in rows if 'stream_level' in r['Name'] or 'slab_level' in r['Name']], key=lambda r: -float(r['TotalDurationNs']))[:8]:
    n = re.sub(r'bnpp::|\(.*', '', r['Name'])
    print("  %-60s %5s calls %8.1f ms  max %7.3f ms" % (n[:60], r['Calls'], float(r['TotalDurationNs']) / 1e6, float(r['MaxNs']) / 1e6))
PY
done
