#!/bin/bash
# Dense split runs (chainsplit.cuh DENSE) against the general addressing
# (BNPP_NO_DENSE=1) on the 32x32 bucket-tree MAR, per-kernel stats; the
# bucket-tree GPU tests first.  (GPU box, repo root)
set -o pipefail
R=$PWD
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bucket_tree.py -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/tree_tests.log 2>&1
rc=$?; tail -2 $R/gpurun_out/tree_tests.log
[ $rc -eq 0 ] || exit $rc
for nd in ${DENSE_SET:-0 1}; do
  OUT=$R/gpurun_out/dense_$nd
  mkdir -p $OUT
  (cd /tmp && BNPP_NO_DENSE=$nd timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 > $OUT/log 2>&1) || { tail -5 $OUT/log; exit 1; }
  echo "== no_dense=$nd"; grep -E '"mar"|"check"' $OUT/log | cut -c1-160
  python3 - $OUT/k_kernel_stats.csv <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:6]:
    n = re.sub(r'bnpp::|\(.*', '', r['Name'])
    print("  %-56s %5s calls %8.1f ms  avg %7.3f ms" % (n[:56], r['Calls'], float(r['TotalDurationNs']) / 1e6, float(r['AverageNs']) / 1e6))
PY
done
