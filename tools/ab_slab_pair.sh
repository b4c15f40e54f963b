set -o pipefail
timeout -k 10 300 ./build/widebw > gpurun_out/widebw.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --no-mar --no-cpu > gpurun_out/ab_pair.log 2>&1 || exit 1
BNPP_NO_SLAB_PAIR=1 timeout -k 10 300 python3 bench.py --no-mar --no-cpu > gpurun_out/ab_nopair.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/parity.log 2>&1
tail -2 gpurun_out/parity.log
cat gpurun_out/widebw.jsonl
for f in ab_pair ab_nopair; do python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][0]); print('$f', d['roofline']['frac'], d['fp64_bucket'])"; done
