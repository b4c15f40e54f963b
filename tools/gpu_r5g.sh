#!/bin/bash
# Round 5: fp32 dense forward split runs two tiles ahead (default build) vs one
# (lib_ahead1), same box, interleaved; identity tests on the default build.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_bucket_tree.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for lib in lib lib_ahead1; do
    BNPP_LIB=$R/bn-pp_amd/$lib/libbnpp.so timeout -k 10 200 python3 -u tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 3 > $OUT/mar_$lib.$i.log 2>&1 || { tail -5 $OUT/mar_$lib.$i.log; exit 1; }
    echo "$lib $i $(grep '"phase": "mar"' $OUT/mar_$lib.$i.log | python3 -c 'import sys,json; print([round(json.loads(l)["wall_ms"],1) for l in sys.stdin])')"
  done
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/mar32 -o mar32 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 > $OUT/mar32.log 2>&1 || exit 1
cd $R
head -4 $(find $OUT/mar32 -name "*kernel_stats.csv") | cut -c1-160
