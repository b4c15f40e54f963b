#!/bin/bash
# Full GPU tests, per-target MAR timing (12x32), then the bench line.  (GPU box, repo root)
R=$PWD
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/gputest.log 2>&1
rc=$?
tail -2 $R/gpurun_out/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest status $rc: stopping"; exit $rc; fi
BNPP_TIMING=1 timeout -k 10 120 python3 -u tools/pertarget_timing.py > $R/gpurun_out/pt.log 2>&1 || exit 1
grep -E "^mar|per-target|build_schedule:|marginals:" $R/gpurun_out/pt.log
timeout -k 10 400 python3 -u bench.py > $R/gpurun_out/bench.log 2>&1
rc2=$?
tail -c 5000 $R/gpurun_out/bench.log
exit $(( rc != 0 ? rc : rc2 ))
