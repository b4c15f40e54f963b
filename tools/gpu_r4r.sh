#!/bin/bash
# Round 4 (r): the N-rank bench path rehearsed on one GPU after the fused
# beliefs and shared reduction levels: two ranks over gloo, a 24x24 MAR with
# 2^16-entry kept sets (so each part's deliveries fuse their beliefs), the
# record printed before the sliced leg.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r4r
mkdir -p $OUT
BNPP_KEEP_LOG2=16 BNPP_BENCH_REHEARSE=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --mar-rows 24 --mar-cols 24 \
  > $OUT/rehearse2.json 2> $OUT/rehearse2.err || { tail -20 $OUT/rehearse2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/rehearse2.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'value', d['value'], 'mar', d['mar']['wall_ms'], 'check', d['mar']['check'])"
grep sliced_mar $OUT/rehearse2.err | cut -c1-300
