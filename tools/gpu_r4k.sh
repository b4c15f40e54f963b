#!/bin/bash
# Round 4: the split-run probe (tools/bwdprobe.hip) and the engine's 32x32 MAR
# kernel stats on the same box.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r4k
mkdir -p $OUT
timeout -k 10 200 $R/build/bwdprobe > $OUT/bwdprobe.jsonl 2>&1 || { tail -5 $OUT/bwdprobe.jsonl; exit 1; }
bash tools/ab_split_r4.sh base > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
