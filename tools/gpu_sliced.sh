#!/bin/bash
# sliced bucket-tree MAR on the GPU box: tests, then the 32x32 projection
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sliced.py tests/test_gpu_bucket_tree.py -x -v --timeout 300 --timeout-method thread > gpurun_out/sliced_tests.log 2>&1 || { tail -40 gpurun_out/sliced_tests.log; exit 1; }
tail -4 gpurun_out/sliced_tests.log
timeout -k 10 900 python3 tools/mar_sliced.py --ranks ${1:-8 4} > gpurun_out/mar_sliced.jsonl 2> gpurun_out/mar_sliced.err || { tail -20 gpurun_out/mar_sliced.err; exit 1; }
cat gpurun_out/mar_sliced.jsonl
