#!/bin/bash
# Round 4 (g): generic-kernel load batching -- full GPU suite, corpus PR phases,
# Munin1 kernel trace, 32x32 MAR kernel stats, bench.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r4g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || exit 1
BNPP_TIMING=1 timeout -k 10 120 python3 -u $R/tools/pr_phases.py Mildew.uai Barley.uai pathfinder.uai Munin1.uai Link.uai noisyor_50_80.uai:noisyor_50_80.uai.evid > $OUT/pr_phases.jsonl 2> $OUT/pr_phases.err || exit 1
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/munin1 -o k --output-format csv -- python3 $R/tools/pr_phases.py Munin1.uai > $OUT/munin1.log 2>&1) || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/mar32 -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 > $OUT/mar32.log 2>&1) || exit 1
