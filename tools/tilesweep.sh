# A/B of the fused bucket kernel variants on the bench shape (one process per variant)
set -e
mkdir -p gpurun_out
for t in 4 8 16; do
  BNPP_MAX_TILE=$t timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_tile$t.log 2>&1
  BNPP_NO_STREAM=1 BNPP_MAX_TILE=$t timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_generic_tile$t.log 2>&1
done
