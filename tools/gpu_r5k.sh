#!/bin/bash
# Round 5: split runs with fewer vector instructions per tile (entries paired
# for packed fp32 arithmetic without re-pairing moves, v_max3 for the running
# max, uniform wave id, scalar-base + 32-bit lane-offset addressing, run state
# through the scalar cache): bucket-tree tests, then fp32 and fp64 32x32 MAR
# with the product build and the previous one (lib_base), kernel traces.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_bucket_tree.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for dt in f32 f64; do
for v in main base; do
  if [ $v = main ]; then unset BNPP_LIB; else export BNPP_LIB=$R/bn-pp_amd/lib_$v/libbnpp.so; fi
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/mar_${dt}_$v -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --dtype $dt --check 1 --reps 2 > $OUT/mar_${dt}_$v.jsonl 2> $OUT/mar_${dt}_$v.err) || { tail -5 $OUT/mar_${dt}_$v.err; exit 1; }
  echo "== $dt $v"; grep -h '"mar"\|check' $OUT/mar_${dt}_$v.jsonl | cut -c1-200
  head -5 $(find $OUT/mar_${dt}_$v -name "*kernel_stats.csv") | cut -c1-160
done
done
