#!/bin/bash
# Round 4: beliefs fused into the backward runs (kChainBel) -- bucket-tree and
# parity tests, then the 32x32 MAR with and without the fusion on one box
# (kernel stats, interleaved).
set -o pipefail
R=$PWD
export TMPDIR=/tmp
OUT=$R/gpurun_out/r4l
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_bucket_tree.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in nofuse fuse nofuse fuse; do
  mkdir -p $OUT/$v
  F=0; [ $v = nofuse ] && F=1
  (cd /tmp && BNPP_NO_BEL_FUSE=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 > $OUT/$v/log 2>&1) || { tail -5 $OUT/$v/log; exit 1; }
  echo "== $v"; grep -E '"mar"|"check"' $OUT/$v/log | cut -c1-220
  python3 - $OUT/$v/k_kernel_stats.csv <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:5]:
    n = re.sub(r'bnpp::|\(.*', '', r['Name'])
    print("  %-52s %5s calls %8.1f ms  avg %7.3f ms" % (n[:52], r['Calls'], float(r['TotalDurationNs']) / 1e6, float(r['AverageNs']) / 1e6))
PY
done
