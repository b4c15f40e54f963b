#!/bin/bash
# Round 4, slab form with outer dims: full GPU suite, default bench line and
# the 32x32 MAR kernel stats.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r4t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/mar32 -o mar32 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 > $OUT/mar32.log 2>&1 || exit 1
cd $R
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'], 'mar warm', d['mar']['wall_ms'], 'cold', d['mar']['cold_wall_ms'], 'fp64 frac', d['fp64_bucket']['frac'])"
grep -E '"mar"' $OUT/mar32.log | cut -c1-140
