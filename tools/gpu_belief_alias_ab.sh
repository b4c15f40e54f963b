set -o pipefail
R=$PWD
OUT=$R/gpurun_out/belab
mkdir -p $OUT
export TMPDIR=/tmp
BNPP_LIB=$R/bn-pp_amd/lib_belalias/libbnpp.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_bucket_tree.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
cd /tmp
for v in base alias; do
  L=$R/bn-pp_amd/lib/libbnpp.so; [ $v = alias ] && L=$R/bn-pp_amd/lib_belalias/libbnpp.so
  BNPP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 0 --reps 2 > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
  grep '"phase": "mar"' $OUT/$v.log | cut -c1-140
  grep "ELi1EEEv\|, 1>(" $OUT/$v/k_kernel_stats.csv | grep "chain_split_kernel<double, 7, 2, 1, true, 1>" | cut -c1-200
done
