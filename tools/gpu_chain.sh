set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bucket_tree.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tree.log 2>&1 || { tail -30 gpurun_out/gpu_tree.log; exit 1; }
tail -2 gpurun_out/gpu_tree.log
timeout -k 10 300 python tools/ve_bench.py --only 32x32 > gpurun_out/ve32.jsonl 2>&1 || { tail -5 gpurun_out/ve32.jsonl; exit 1; }
tail -1 gpurun_out/ve32.jsonl | cut -c1-200
bash tools/prof_mar32.sh || exit 1
grep phase gpurun_out/prof_mar32/mar32.log | cut -c1-200
