#!/bin/bash
# Round 4: fused beliefs with the forward-message loads issued before the next
# tile's row loads -- bucket-tree tests, then the 32x32 MAR fused / unfused on
# one box, interleaved, with the fused runs' own durations from the trace.
set -o pipefail
R=$PWD
export TMPDIR=/tmp
OUT=$R/gpurun_out/r4q
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_bucket_tree.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in nofuse fuse nofuse fuse; do
  mkdir -p $OUT/$v
  F=0; [ $v = nofuse ] && F=1
  (cd /tmp && BNPP_NO_BEL_FUSE=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 > $OUT/$v/log 2>&1) || { tail -5 $OUT/$v/log; exit 1; }
  echo "== $v"; grep -E '"mar"' $OUT/$v/log | cut -c1-150
  python3 - $OUT/$v/k_kernel_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = sorted((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows if 'chain_split_kernel<8, 2, 1' in r['Kernel_Name'])
f = sorted((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows if 'chain_split_kernel<8, 1, 0' in r['Kernel_Name'])
b = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows if 'bucket_level_kernel<float, 2, 4, 1>' in r['Kernel_Name']]
b = [x for x in b if x > 1]
print("  fwd %d avg %.3f | bwd %d avg %.3f, slowest 78 avg %.3f, rest avg %.3f | belief passes %d avg %.3f" % (
    len(f), sum(f) / len(f), len(d), sum(d) / len(d), sum(d[-78:]) / 78, sum(d[:-78]) / (len(d) - 78), len(b), sum(b) / max(1, len(b))))
PY
done
