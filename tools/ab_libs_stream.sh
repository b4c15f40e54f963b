#!/bin/bash
# 32x32 bucket-tree MAR per library variant (base = bn-pp_amd/lib, else
# bn-pp_amd/lib_<name>): wall and the stream / slab level kernels' totals.
# usage: tools/ab_libs_stream.sh base u32 ...
set -o pipefail
R=$PWD
export TMPDIR=/tmp
for v in "$@"; do
  if [ $v = base ]; then L=$R/bn-pp_amd/lib/libbnpp.so; else L=$R/bn-pp_amd/lib_$v/libbnpp.so; fi
  OUT=$R/gpurun_out/abs_$v
  mkdir -p $OUT
  (cd /tmp && BNPP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 > $OUT/log 2>&1) || { tail -5 $OUT/log; exit 1; }
  echo "== $v"; grep -E '"mar"|"check"' $OUT/log | cut -c1-150
  python3 - $OUT/k_kernel_stats.csv <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows) / 1e6
def s(key): return sum(float(r['TotalDurationNs']) for r in rows if key in r['Name']) / 1e6
print("  all kernels %.1f ms, stream_level %.1f ms, slab_level %.1f ms" % (tot, s('stream_level'), s('slab_level')))
for r in sorted([r for r in rows if 'stream_level' in r['Name']], key=lambda r: -float(r['TotalDurationNs']))[:6]:
    n = re.sub(r'bnpp::|\(.*', '', r['Name'])
    print("  %-60s %5s calls %8.1f ms  max %7.3f ms" % (n[:60], r['Calls'], float(r['TotalDurationNs']) / 1e6, float(r['MaxNs']) / 1e6))
PY
done
