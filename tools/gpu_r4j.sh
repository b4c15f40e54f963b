#!/bin/bash
# Round 4: workgroup-contiguous row traffic in the split runs -- bucket-tree
# parity tests, then the 32x32 MAR kernel stats against the previous library
# (bn-pp_amd/lib_old) on the same box, interleaved.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r4j
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_bucket_tree.py > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/ab_split_r4.sh old base old base > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
