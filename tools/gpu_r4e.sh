#!/bin/bash
# Round 4 (e): corpus PR phase split after the source cache; kernel trace of
# Munin1's PR (which kernel holds its 4 ms of device time).
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r4e
mkdir -p $OUT
export TMPDIR=/tmp
BNPP_TIMING=1 timeout -k 10 120 python3 -u $R/tools/pr_phases.py Mildew.uai Barley.uai pathfinder.uai Munin1.uai Link.uai noisyor_50_80.uai:noisyor_50_80.uai.evid > $OUT/pr_phases.jsonl 2> $OUT/pr_phases.err || exit 1
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/munin1 -o k --output-format csv -- python3 $R/tools/pr_phases.py Munin1.uai > $OUT/munin1.log 2>&1) || exit 1
timeout -k 10 200 python3 -u $R/tools/config4_bench.py > $OUT/config4_bench.jsonl 2> $OUT/config4_bench.err || exit 1
