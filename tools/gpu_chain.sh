set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bucket_tree.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tree.log 2>&1 || { tail -30 gpurun_out/gpu_tree.log; exit 1; }
tail -3 gpurun_out/gpu_tree.log
bash tools/prof_mar32.sh || exit 1
tail -4 gpurun_out/prof_mar32/mar32.log
