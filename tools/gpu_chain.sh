set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bucket_tree.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tree.log 2>&1 || { tail -30 gpurun_out/gpu_tree.log; exit 1; }
tail -3 gpurun_out/gpu_tree.log
timeout -k 10 300 python -u tools/mar_grid.py --rows 32 --cols 32 --check 2 > gpurun_out/mar32_chain.jsonl 2>&1 || { tail -5 gpurun_out/mar32_chain.jsonl; exit 1; }
cat gpurun_out/mar32_chain.jsonl
