#!/bin/bash
# kernel trace of rank 0's share of the 8-rank sliced 32x32 MAR (loopback, no copies)
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/prof_sliced
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o sl --output-format csv -- python3 $R/tools/mar_sliced.py --ranks ${1:-8} --reps 2 > $OUT/run.log 2>&1
