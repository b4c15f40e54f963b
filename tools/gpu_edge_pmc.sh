#!/bin/bash
# PMC traffic of the 32x32 MAR's edge buckets (slab / stream level kernels).
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/edge
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 1 > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 1 > $OUT/write.log 2>&1 || exit 1
cd $R
python3 tools/edge_traffic.py $(find $OUT/fetch -name "*counter_collection.csv") $(find $OUT/write -name "*counter_collection.csv") > $OUT/edge_traffic.json || exit 1
cat $OUT/edge_traffic.json
