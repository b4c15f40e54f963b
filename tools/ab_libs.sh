# A/B alternative library builds on the bench bucket and the 32x32 sweep (experiments)
set -e
mkdir -p gpurun_out
for v in base w5 w6; do
  if [ $v = base ]; then L=$PWD/bn-pp_amd/lib/libbnpp.so; else L=$PWD/bn-pp_amd/lib_$v/libbnpp.so; fi
  BNPP_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-mar > gpurun_out/ab_$v.log 2>&1
  BNPP_LIB=$L timeout -k 10 300 python tools/ve_bench.py --only 32x32 > gpurun_out/ab32_$v.jsonl 2>&1
done
