#!/bin/bash
# Round-4 rocprofv3 evidence (GPU box, repo root): bench kernel trace+stats,
# FETCH_SIZE / WRITE_SIZE (separate passes) of the f32 and the f64 bench
# bucket, the 32x32 MAR kernel stats and its split runs' SQ counters.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/prof4
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="--no-cpu --no-mar --no-fp64"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 $B > $OUT/trace.log 2>&1 || exit 1
for DT in f32 f64; do
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$DT -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --dtype $DT $B > $OUT/fetch_$DT.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_$DT -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --dtype $DT $B > $OUT/write_$DT.log 2>&1 || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/mar32 -o mar32 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 > $OUT/mar32.log 2>&1 || exit 1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P -d $OUT/sq$i -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 1 > $OUT/sq$i.log 2>&1 || exit 1
done
cd $R
python3 tools/pmc_traffic.py $(find $OUT/fetch_f32 -name "*counter_collection.csv") $(find $OUT/write_f32 -name "*counter_collection.csv") > $OUT/traffic_f32.json || exit 1
python3 tools/pmc_traffic.py --dtype f64 --kernel "slab_single_kernel<double" $(find $OUT/fetch_f64 -name "*counter_collection.csv") $(find $OUT/write_f64 -name "*counter_collection.csv") > $OUT/traffic_f64.json || exit 1
