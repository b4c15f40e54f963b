#!/bin/bash
# Round 5: on-demand VMM arena mapping, fp64 split runs.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_bucket_tree.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python3 -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
m=d['mar']; print('mar warm', m['wall_ms'], 'cold', m['cold_wall_ms']); print('cold phases', json.dumps(m['phases_ms']['cold']))"
for v in 0 1; do
  BNPP_NO_VMM=$v timeout -k 10 200 python3 -u tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 > $OUT/mar_vmm$v.log 2>&1 || { tail -5 $OUT/mar_vmm$v.log; exit 1; }
  echo "NO_VMM=$v"; grep -E '"phase": "mar"' $OUT/mar_vmm$v.log | python3 -c "import sys,json
for l in sys.stdin: d=json.loads(l); print(d['rep'], round(d['wall_ms'],1), {k: round(v,1) for k,v in d['phases'].items()})"
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/mar64 -o mar64 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 1 --reps 1 > $OUT/mar64.log 2>&1 || { tail -5 $OUT/mar64.log; exit 1; }
cd $R
grep -E '"phase"' $OUT/mar64.log | cut -c1-300
head -8 $(find $OUT/mar64 -name "*kernel_stats.csv") | cut -c1-160
