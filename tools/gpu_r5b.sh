#!/bin/bash
# Round 5: the VMM-mapped arena.  The 32x32 tree test (VMM vs hipMalloc
# identity), then the bench right after it (the driver's order: a process
# that freed ~250 GB just before), then a cold MAR in a fresh process with
# and without VMM.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_bucket_tree.py -k "32x32 or fused_beliefs or split_runs" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python3 -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
m=d['mar']; print('mar warm', m['wall_ms'], 'cold', m['cold_wall_ms']); print('cold phases', json.dumps(m['phases_ms']['cold'])); print('warm phases', json.dumps(m['phases_ms']['warm']))"
for v in 0 1 0; do
  BNPP_NO_VMM=$v timeout -k 10 200 python3 -u tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 > $OUT/mar_vmm$v.log 2>&1 || { tail -5 $OUT/mar_vmm$v.log; exit 1; }
  echo "NO_VMM=$v"; grep -E '"phase": "mar"' $OUT/mar_vmm$v.log | python3 -c "import sys,json
for l in sys.stdin: d=json.loads(l); print(d[\"rep\"], round(d[\"wall_ms\"],1), {k: round(v,1) for k,v in d[\"phases\"].items()})"
done
