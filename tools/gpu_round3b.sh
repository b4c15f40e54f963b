#!/bin/bash
# Full GPU tests, then the dense-run A/B on the 32x32 MAR, then per-target MAR
# timing at 12x32 (dedup on / off).  (GPU box, repo root)
R=$PWD
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/gputest.log 2>&1
rc=$?
tail -3 $R/gpurun_out/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest status $rc: stopping"; exit $rc; fi
DENSE_SET="0 1" timeout -k 10 700 bash tools/ab_dense.sh > $R/gpurun_out/ab_dense.log 2>&1 || { tail -5 $R/gpurun_out/ab_dense.log; exit 1; }
grep -v "^\.\|passed" $R/gpurun_out/ab_dense.log
for nd in 0 1; do
  BNPP_NO_DEDUP=$nd BNPP_TIMING=1 timeout -k 10 120 python3 -u tools/pertarget_timing.py > $R/gpurun_out/pt_$nd.log 2>&1 || exit 1
  echo "== no_dedup=$nd"; grep -E "^mar|schedules|plans |marginals:" $R/gpurun_out/pt_$nd.log
done
exit $rc
