#!/bin/bash
# Round 4 (s): fp64 slab bucket, paired lanes splitting the big loads
# (slab_load_big_pair) vs both loading all (bn-pp_amd/lib_old), interleaved.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r4s
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in old new old new old new; do
  LIB=$R/bn-pp_amd/lib/libbnpp.so; [ $v = old ] && LIB=$R/bn-pp_amd/lib_old/libbnpp.so
  BNPP_LIB=$LIB timeout -k 10 200 python3 -u bench.py --dtype f64 --no-cpu --no-mar --no-fp64 --steps 30 --warmup 3 > $OUT/$v.json 2> $OUT/$v.err || { tail -5 $OUT/$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1])
print('$v', 'kernel_ms %.4f frac %.4f spot %s' % (d['roofline']['kernel_ms'], d['roofline']['frac'], d['spot_check_exact']))"
done
