#!/bin/bash
# Round-3 probe of the 32x32 MAR (run on the GPU box from the repo root):
#  1. cold vs warm phase split in a fresh process (BNPP_TIMING)
#  2. kernel trace of a cold + warm call (where the cold call's extra time goes)
#  3. FETCH_SIZE and WRITE_SIZE of the split chain runs (separate --pmc passes)
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/cold
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
BNPP_TIMING=1 timeout -k 10 240 python3 -u $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 3 > $OUT/timing.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o mar --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o mar --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 1 > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o mar --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 1 > $OUT/write.log 2>&1 || exit 1
cd $R
python3 tools/trace_calls.py $(find $OUT/trace -name "*kernel_trace.csv") > $OUT/calls.json || exit 1
python3 tools/pmc_kernels.py $(find $OUT/fetch -name "*counter_collection.csv") $(find $OUT/write -name "*counter_collection.csv") > $OUT/pmc_mar32.json
