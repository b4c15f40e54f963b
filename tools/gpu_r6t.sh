# Deferred belief sum in the fused backward runs (chain_split_kernel MODE 1):
# bucket-tree tests, then the 32x32 fp32 MAR kernel stats (belief runs' time).
set -o pipefail
R=$PWD
O=$R/gpurun_out/r6t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bucket_tree.py tests/test_gpu_sliced.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/mar32 -o mar32 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 2 --reps 3 > $O/mar32.jsonl 2> $O/mar32.err || { tail -20 $O/mar32.err; exit 1; }
cd $R
grep -o '"wall_ms": [0-9.]*' $O/mar32.jsonl | tr '\n' ' '; echo
head -5 $(find $O/mar32 -name "*kernel_stats.csv") | cut -c1-160
echo ok
# fp64 32x32 MAR: the product build (separate fp64 belief passes) and the
# BNPP_F64_BEL8 variant (fused fp64 belief runs of 8), warm walls
for lib in lib lib_bel8; do
  BNPP_LIB=$R/bn-pp_amd/$lib/libbnpp.so timeout -k 10 300 python3 -u tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 1 --reps 3 > $O/mar64_$lib.jsonl 2> $O/mar64_$lib.err || { tail -5 $O/mar64_$lib.err; exit 1; }
  echo "f64 $lib: $(grep -o '"wall_ms": [0-9.]*' $O/mar64_$lib.jsonl | tr '\n' ' ') $(grep -o '"abs_err": [0-9.e-]*' $O/mar64_$lib.jsonl | head -1)"
done
echo ok2
