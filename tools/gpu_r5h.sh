#!/bin/bash
# Round 5: generic gather kernel without the per-input load waits (broadcast
# values no longer copied before use, dims pool through the scalar cache):
# Munin1's kernel trace, then the parity tests that run the generic kernels.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5h
mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/munin1 -o k --output-format csv -- python3 $R/tools/pr_phases.py Munin1.uai > $OUT/munin1.log 2>&1) || { tail -5 $OUT/munin1.log; exit 1; }
head -6 $(find $OUT/munin1 -name "*kernel_stats.csv") | cut -c1-200
cat $OUT/munin1.log | cut -c1-300
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_config4.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
