# parity tests + bench bucket + 32x32 PR + 32x32 MAR (one GPU call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-mar > gpurun_out/bq.log 2>&1 || { tail -5 gpurun_out/bq.log; exit 1; }
python -c "
import json; l=[x for x in open('gpurun_out/bq.log') if x.startswith('{')]; d=json.loads(l[-1]); print('bench', d['roofline']['kernel_ms'], round(d['roofline']['frac'],4))"
timeout -k 10 300 python tools/ve_bench.py --only 32x32 > gpurun_out/ve32.jsonl 2>&1 || { tail -5 gpurun_out/ve32.jsonl; exit 1; }
tail -1 gpurun_out/ve32.jsonl
BNPP_TIMING=1 timeout -k 10 300 python tools/mar_grid.py --rows 32 --cols 32 --check 1 > gpurun_out/mar32.log 2>&1 || { tail -5 gpurun_out/mar32.log; exit 1; }
grep -E "tree marginals|phase" gpurun_out/mar32.log
