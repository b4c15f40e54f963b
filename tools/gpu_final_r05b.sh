#!/bin/bash
# Round-5 closing evidence, part B: the 32x32 MAR kernel stats (fp32 and
# fp64), the split runs' HBM traffic (separate FETCH_SIZE / WRITE_SIZE
# passes), config 4 against the reference pinned to one core, and the
# self-launched two-rank rehearsal.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/final5h
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/mar32 -o mar32 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 2 --reps 2 > $OUT/mar32.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/mfetch -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 1 > $OUT/mfetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/mwrite -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 1 > $OUT/mwrite.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/mar64 -o mar64 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 1 --reps 2 > $OUT/mar64.log 2>&1 || exit 1
cd $R
python3 tools/mar_traffic.py $(find $OUT/mfetch -name "*counter_collection.csv") $(find $OUT/mwrite -name "*counter_collection.csv") > $OUT/mar_traffic.json || exit 1
grep -E '"phase": "(mar|check)"' $OUT/mar32.log | cut -c1-160
grep -E '"phase": "(mar|check)"' $OUT/mar64.log | cut -c1-160
timeout -k 10 600 python3 -u tools/config4_bench.py > $OUT/config4.jsonl 2> $OUT/config4.err || { tail -20 $OUT/config4.err; exit 1; }
BNPP_BENCH_REHEARSE=1 timeout -k 10 400 python3 -u bench.py --gpus 2 --no-cpu --no-mar-f64 --mar-rows 16 --mar-cols 16 > $OUT/rehearse2.json 2> $OUT/rehearse2.err || { tail -20 $OUT/rehearse2.err; exit 1; }
cat $OUT/config4.jsonl | cut -c1-600
