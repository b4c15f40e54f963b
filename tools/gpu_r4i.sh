#!/bin/bash
# Round 4 (i): the N-rank bench path rehearsed on one GPU (two ranks over
# gloo, BNPP_BENCH_REHEARSE=1, 16x16 MAR: record printed before the sliced leg,
# sliced leg on stderr), the GPU suite (job cache), then the default bench.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r4i
mkdir -p $OUT
BNPP_BENCH_REHEARSE=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --mar-rows 16 --mar-cols 16 \
  > $OUT/rehearse2.json 2> $OUT/rehearse2.err || exit 1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
