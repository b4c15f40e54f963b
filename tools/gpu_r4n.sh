#!/bin/bash
# Round 4: full GPU suite after the fused beliefs, then the default bench line.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r4n
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'], 'mar warm', d['mar']['wall_ms'], 'cold', d['mar']['cold_wall_ms'], 'fp64 frac', d['fp64_bucket']['frac'])"
