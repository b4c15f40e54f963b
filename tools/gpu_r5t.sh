#!/bin/bash
# Round 5: stream kernels reading the dims pool through the scalar cache:
# parity tests, then PR timings of the corpus (stream-form buckets) and the
# 32x32 MAR's stream kernels, product build against lib_base.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_config4.py tests/test_gpu_bucket_tree.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in main base; do
  if [ $v = main ]; then unset BNPP_LIB; else export BNPP_LIB=$R/bn-pp_amd/lib_$v/libbnpp.so; fi
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/pr_$v -o k --output-format csv -- python3 $R/tools/pr_phases.py Munin1.uai Munin2.uai:Munin2.uai.evid Pigs.uai Barley.uai Mildew.uai Link.uai > $OUT/pr_$v.log 2>&1) || { tail -5 $OUT/pr_$v.log; exit 1; }
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/mar_$v -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 1 > $OUT/mar_$v.log 2>&1) || { tail -5 $OUT/mar_$v.log; exit 1; }
  echo "== $v"; grep '^{' $OUT/pr_$v.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  %-10s %.3f ms' % (d['model'], d['wall_ms_median']))"
  grep -h "stream_level" $(find $OUT/pr_$v -name "*kernel_stats.csv") | cut -c1-150 | head -6
  grep -h "stream_level" $(find $OUT/mar_$v -name "*kernel_stats.csv") | cut -c1-150 | head -6
done
