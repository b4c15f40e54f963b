#!/bin/bash
# Round 5 first GPU call: the GPU suite, the default bench line, and the
# self-launched two-rank rehearsal (gloo, both ranks on the one GPU).
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
BNPP_BENCH_REHEARSE=1 timeout -k 10 400 python3 -u bench.py --gpus 2 --no-cpu --mar-rows 16 --mar-cols 16 > $OUT/rehearse2.json 2> $OUT/rehearse2.err || { tail -20 $OUT/rehearse2.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'], 'mar warm', d['mar']['wall_ms'], 'cold', d['mar']['cold_wall_ms'], 'fp64 frac', d['fp64_bucket']['frac'])
print('secondary', json.dumps(d['mar']['secondary']))
r=json.loads(open('$OUT/rehearse2.json').read().strip().splitlines()[-1])
print('rehearse n_gpus', r['n_gpus'], r['backend'], 'sliced', json.dumps(r['mar'].get('sliced')))"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/mar32 -o mar32 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 > $OUT/mar32.log 2>&1 || exit 1
cd $R
grep -E '"mar"|wall' $OUT/mar32.log | cut -c1-200
head -12 $(find $OUT/mar32 -name "*kernel_stats.csv") | cut -c1-200
