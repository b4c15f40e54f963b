#!/bin/bash
# Loopy BP on the GPU box: flood tests, single vs flood timings, flood kernel trace.
mkdir -p gpurun_out/bpprof2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bp_tests.log 2>&1
rc=$?
tail -2 gpurun_out/bp_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/bp_modes.py > gpurun_out/bp_modes.jsonl 2>&1 || exit 1
cat gpurun_out/bp_modes.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/bpprof2 -o bp --output-format csv -- python3 tools/bp_prof.py 128 > gpurun_out/bpprof2/log 2>&1 || exit 1
grep ising gpurun_out/bpprof2/log
head -8 gpurun_out/bpprof2/bp_kernel_stats.csv
exit $rc
