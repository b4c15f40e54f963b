#!/bin/bash
# GPU tests then the bench (run on the GPU box from the repo root).  A test
# failure (pytest status 1) still runs the bench; a fault, abort, segfault or
# time limit (any other status) ends the call.
R=$PWD
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $R/gpurun_out/gputest.log 2>&1
rc=$?
tail -4 $R/gpurun_out/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest status $rc: stopping"; exit $rc; fi
timeout -k 10 400 python3 -u bench.py > $R/gpurun_out/bench.log 2>&1
rc2=$?
tail -c 4000 $R/gpurun_out/bench.log
exit $(( rc != 0 ? rc : rc2 ))
