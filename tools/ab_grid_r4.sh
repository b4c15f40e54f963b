#!/bin/bash
# Round 4: workgroups per CU for the generic (gather) kernels -- Munin1 PR
# kernel stats at BNPP_GRID_PER_CU = 3 (default), 8, 16, 0 (flat grid).
set -o pipefail
R=$PWD
export TMPDIR=/tmp
for g in 3 8 16 0; do
  OUT=$R/gpurun_out/grid4/g$g
  mkdir -p $OUT
  (cd /tmp && BNPP_GRID_PER_CU=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o k --output-format csv -- python3 $R/tools/pr_phases.py Munin1.uai Link.uai Barley.uai > $OUT/log 2>&1) || exit 1
  echo "== per_cu $g"; cat $OUT/log | grep model | cut -c1-120
  python3 - $OUT/k_kernel_stats.csv <<'PY'
import csv, re, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:4]:
    print("  %-60s %5s calls avg %7.3f ms" % (re.sub(r'bnpp::|\(.*', '', r['Name'])[:60], r['Calls'], float(r['AverageNs']) / 1e6))
PY
done
