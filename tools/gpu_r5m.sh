#!/bin/bash
# Round 5: odd-card stream buckets on the generic whole-dim tiles: Munin1 PR
# kernel traces with the tuning build (lib_knobs) with and without
# BNPP_ODD_STREAM=1 (the stream form kept), then the parity tests.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5m
mkdir -p $OUT
export TMPDIR=/tmp
export BNPP_LIB=$R/bn-pp_amd/lib_knobs/libbnpp.so
for v in generic stream; do
  if [ $v = stream ]; then export BNPP_ODD_STREAM=1; else unset BNPP_ODD_STREAM; fi
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/munin1_$v -o k --output-format csv -- python3 $R/tools/pr_phases.py Munin1.uai Munin2.uai:Munin2.uai.evid Munin3.uai Munin4.uai > $OUT/munin1_$v.log 2>&1) || { tail -5 $OUT/munin1_$v.log; exit 1; }
  echo "== $v"; grep '^{' $OUT/munin1_$v.log | cut -c1-120
  head -8 $(find $OUT/munin1_$v -name "*kernel_stats.csv") | cut -c1-160
done
unset BNPP_LIB BNPP_ODD_STREAM
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_config4.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
