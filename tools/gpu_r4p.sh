#!/bin/bash
# Round 4: kept-table reductions at free levels (one launch per depth instead
# of one per bucket) -- bucket-tree tests, then the 32x32 MAR with and without
# (BNPP_NO_FREE_REDUCE=1) on one box, interleaved.
set -o pipefail
R=$PWD
export TMPDIR=/tmp
OUT=$R/gpurun_out/r4p
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_bucket_tree.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in seq free seq free; do
  mkdir -p $OUT/$v
  F=0; [ $v = seq ] && F=1
  (cd /tmp && BNPP_NO_FREE_REDUCE=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 > $OUT/$v/log 2>&1) || { tail -5 $OUT/$v/log; exit 1; }
  echo "== $v"; grep -E '"mar"' $OUT/$v/log | cut -c1-150
  python3 - $OUT/$v/k_kernel_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
small = [r for r in rows if int(r['End_Timestamp']) - int(r['Start_Timestamp']) < 50e3]
print("  kernels %d, small %d, small total %.1f ms" % (len(rows), len(small), sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in small) / 1e6))
PY
done
