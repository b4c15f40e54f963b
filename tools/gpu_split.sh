#!/bin/bash
# Split chain runs on the GPU box: identity tests (bucket tree), then the 32x32
# MAR under a kernel trace, then the BP script.  (repo root)
set -o pipefail
mkdir -p gpurun_out/split
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bucket_tree.py -x -q --timeout 300 --timeout-method thread > gpurun_out/split/tests.log 2>&1 || { tail -30 gpurun_out/split/tests.log; exit 1; }
tail -2 gpurun_out/split/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/split -o k --output-format csv -- python3 tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 3 > gpurun_out/split/mar.log 2>&1 || { tail -5 gpurun_out/split/mar.log; exit 1; }
grep -E '"mar"|"check"' gpurun_out/split/mar.log | cut -c1-200
head -8 gpurun_out/split/k_kernel_stats.csv | cut -c1-200
bash tools/gpu_bp.sh
