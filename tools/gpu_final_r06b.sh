#!/bin/bash
# Round-6 closing evidence, part B: the 32x32 MAR kernel stats (fp32, fp64)
# with the deferred belief sum, and the self-launched two-rank rehearsal of
# the N-rank bench (gloo, sliced MAR from two ranks, CPU baseline).
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${FINAL_OUT:-final6b}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/mar32 -o mar32 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 2 --reps 3 > $OUT/mar32.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/mar64 -o mar64 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 1 --reps 3 > $OUT/mar64.log 2>&1 || exit 1
cd $R
grep -o '"wall_ms": [0-9.]*' $OUT/mar32.log | tr '\n' ' '; echo
grep -o '"wall_ms": [0-9.]*' $OUT/mar64.log | tr '\n' ' '; echo
BNPP_BENCH_REHEARSE=1 timeout -k 10 500 python3 -u bench.py --gpus 2 --no-mar-f64 --mar-rows 16 --mar-cols 16 > $OUT/rehearse2.json 2> $OUT/rehearse2.err || { tail -20 $OUT/rehearse2.err; exit 1; }
head -4 $(find $OUT/mar32 -name "*kernel_stats.csv") | cut -c1-160
head -4 $(find $OUT/mar64 -name "*kernel_stats.csv") | cut -c1-160
python3 -c "
import json
d=json.loads(open('$OUT/rehearse2.json').read().strip().splitlines()[-1])
print('rehearse2', d['n_gpus'], d['backend'], 'cpu_baseline' in d and d['cpu_baseline'] is not None, {k: d['mar'].get(k) for k in ('scheme', 'wall_ms')}, d['mar'].get('sliced', {}).get('ok') if isinstance(d['mar'].get('sliced'), dict) else None, d.get('checksum_ok'))"
