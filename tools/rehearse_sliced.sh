#!/bin/bash
# bench.py's N-rank path (segment MAR + sliced MAR) rehearsed on one GPU over gloo
set -o pipefail
mkdir -p gpurun_out
for N in 2 4; do
  BNPP_BENCH_REHEARSE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29600 + N)) bench.py --gpus $N --steps 3 --warmup 1 --mar-rows 16 --mar-cols 16 --no-fp64 > gpurun_out/rehearse_$N.log 2>&1 || { tail -30 gpurun_out/rehearse_$N.log; exit 1; }
  grep '^{' gpurun_out/rehearse_$N.log | tail -1 > gpurun_out/rehearse_$N.json
  python3 -c "import json; d=json.load(open('gpurun_out/rehearse_$N.json')); print($N, json.dumps(d['mar'].get('sliced')), d['mar']['wall_ms'])"
done
