# A/B: the arena base aligned to 32 MiB (hipMalloc's own), 1 GiB, 4 GiB
# (BNPP_ARENA_ALIGN_MB in a -DBNPP_TUNING_KNOBS build); 32x32 MAR fp64 and fp32, warm.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r6r; mkdir -p $O
for dt in f64 f32; do
for a in 0 1024 4096 0; do
  BNPP_LIB=$R/bn-pp_amd/lib_knobs/libbnpp.so BNPP_ARENA_ALIGN_MB=$a BNPP_TIMING=1 timeout -k 10 300 python3 -u tools/mar_grid.py --rows 32 --cols 32 --dtype $dt --check 0 --reps 3 > $O/${dt}_$a.jsonl 2> $O/${dt}_$a.err || exit 1
  echo "$dt align $a MB: $(grep -o '"wall_ms": [0-9.]*' $O/${dt}_$a.jsonl | tr '\n' ' ') $(grep -o 'at 0x[0-9a-f]*' $O/${dt}_$a.err | head -1)"
done
done
echo ok
