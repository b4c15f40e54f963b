#!/bin/bash
# Round 5: the default bench line (now with the fp64 32x32 MAR) and config 4
# with first-call GPU times beside the reference pinned to one core.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
m=d['mar']; print('value', d['value'], 'frac', d['roofline']['frac'], 'mar warm', m['wall_ms'], 'cold', m['cold_wall_ms'], 'fp64 frac', d['fp64_bucket']['frac'])
f=d['mar_f64']; print('mar_f64 warm', f['wall_ms'], 'cold', f['cold_wall_ms'], 'check', json.dumps(f.get('check')))
print('secondary', json.dumps(m['secondary']))"
timeout -k 10 600 python3 -u tools/config4_bench.py > $OUT/config4.jsonl 2> $OUT/config4.err || { tail -20 $OUT/config4.err; exit 1; }
cat $OUT/config4.jsonl
