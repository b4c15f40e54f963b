#!/bin/bash
# Round-6 closing evidence, part A (GPU box, repo root): the GPU suite, smoke,
# the default bench line (as the driver runs them) and the bench kernel's trace.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${FINAL_OUT:-final6a}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-mar --no-fp64 > $OUT/trace.log 2>&1 || exit 1
cd $R
python3 -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
m=d['mar']; f=d['mar_f64']
print('value', d['value'], 'frac', d['roofline']['frac'], 'kernel_ms', d['roofline']['kernel_ms'], 'ok', d['checksum_ok'])
print('mar warm', m['wall_ms'], 'cold', m['cold_wall_ms'], 'vs fp64', m.get('check_vs_fp64'))
print('f64 warm', f['wall_ms'], 'cold', f['cold_wall_ms'], '| fp64 bucket frac', d['fp64_bucket']['frac'])
print('secondary', {k: m['secondary'].get(k) for k in ('instance', 'reference_cpu_ms', 'ok')})"
head -3 $(find $OUT/trace -name "*kernel_stats.csv") | cut -c1-180
