#!/bin/bash
# Round 5: generic gather kernel, branch-free odd tiles + 32-bit offsets +
# scalar-cache descriptors: Munin1 kernel trace (product build and the
# branchy-odd-tile variant lib_branchy), then the whole GPU suite.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r5i
mkdir -p $OUT
export TMPDIR=/tmp
for v in main branchy; do
  if [ $v = main ]; then unset BNPP_LIB; else export BNPP_LIB=$R/bn-pp_amd/lib_$v/libbnpp.so; fi
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/munin1_$v -o k --output-format csv -- python3 $R/tools/pr_phases.py Munin1.uai Munin2.uai:Munin2.uai.evid Pigs.uai Barley.uai > $OUT/munin1_$v.log 2>&1) || { tail -5 $OUT/munin1_$v.log; exit 1; }
  echo "== $v"; head -6 $(find $OUT/munin1_$v -name "*kernel_stats.csv") | cut -c1-200
done
unset BNPP_LIB
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
