#!/bin/bash
# Round-4 closing SQ counters of the split runs (two --pmc passes, one MAR call each).
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/sq4
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P -d $OUT/sq$i -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 1 > $OUT/sq$i.log 2>&1 || exit 1
done
cd $R
python3 tools/sq_summary.py $(find $OUT/sq1 -name "*counter_collection.csv") $(find $OUT/sq2 -name "*counter_collection.csv") > $OUT/sq.json || exit 1
head -c 1500 $OUT/sq.json
