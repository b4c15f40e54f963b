# Same-box A/B of the fused belief runs' sum placement: product build (one
# tile late) against lib_early (-DBNPP_BEL_SUM_LATE=0, the round-5 placement),
# alternating, 32x32 fp32 MAR kernel stats.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r6x; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for i in 1 2; do
for lib in lib lib_early; do
  BNPP_LIB=$R/bn-pp_amd/$lib/libbnpp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${lib}_$i -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 3 > $O/${lib}_$i.jsonl 2> $O/${lib}_$i.err || { tail -5 $O/${lib}_$i.err; exit 1; }
  f=$(find $O/${lib}_$i -name "*kernel_stats.csv")
  echo "$lib $i: walls $(grep -o '"wall_ms": [0-9.]*' $O/${lib}_$i.jsonl | cut -d' ' -f2 | tr '\n' ' ') | $(grep -E 'chain_split_kernel<float, 8, (1, 0, true, 0|2, 1, true, 0|2, 1, true, 1)>' $f | awk -F'",' '{print $2}' | awk -F, '{printf "%.3f ms  ", $3/1e6}')"
done
done
echo ok
