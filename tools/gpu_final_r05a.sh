#!/bin/bash
# Round-5 closing evidence, part A (GPU box, repo root): the GPU suite, the
# default bench line, the bench kernel's trace and its HBM traffic (FETCH_SIZE /
# WRITE_SIZE in separate --pmc passes, fp32 and fp64).
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/final5i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cd /tmp
B="--no-cpu --no-mar --no-fp64"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 $B > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $B > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $B > $OUT/write.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch64 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --dtype f64 $B > $OUT/fetch64.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write64 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --dtype f64 $B > $OUT/write64.log 2>&1 || exit 1
cd $R
python3 tools/pmc_traffic.py $(find $OUT/fetch -name "*counter_collection.csv") $(find $OUT/write -name "*counter_collection.csv") > $OUT/traffic_f32.json || exit 1
python3 tools/pmc_traffic.py --dtype f64 $(find $OUT/fetch64 -name "*counter_collection.csv") $(find $OUT/write64 -name "*counter_collection.csv") > $OUT/traffic_f64.json || exit 1
python3 -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
m=d['mar']; f=d['mar_f64']
print('value', d['value'], 'frac', d['roofline']['frac'], 'kernel_ms', d['roofline']['kernel_ms'])
print('mar warm', m['wall_ms'], 'cold', m['cold_wall_ms'], '| f64 warm', f['wall_ms'], 'cold', f['cold_wall_ms'], '| fp64 bucket frac', d['fp64_bucket']['frac'])
for k in ('traffic_f32', 'traffic_f64'):
    t=json.load(open('$OUT/%s.json' % k)); print(k, t['hbm_bytes_per_launch'], t['algorithmic_bytes_per_launch'])"
head -3 $(find $OUT/trace -name "*kernel_stats.csv") | cut -c1-180
