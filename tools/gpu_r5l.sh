#!/bin/bash
# Round 5: the whole GPU suite (with the 32/64-bit offset identity test), then
# Munin1's PR phases and kernel trace with the product build.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
BNPP_TIMING=1 timeout -k 10 120 python3 -u tools/pr_phases.py Munin1.uai Mildew.uai Barley.uai Pigs.uai > $OUT/pr_phases.jsonl 2> $OUT/pr_phases.err || exit 1
cut -c1-300 $OUT/pr_phases.jsonl
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/munin1 -o k --output-format csv -- python3 $R/tools/pr_phases.py Munin1.uai > $OUT/munin1.log 2>&1) || exit 1
head -8 $(find $OUT/munin1 -name "*kernel_stats.csv") | cut -c1-200
