# Pairwise (successive sum_out) belief sums: fused runs and separate passes.
# Bucket-tree and sliced GPU tests, then 32x32 MAR fp32 / fp64 kernel stats.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r6w; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_bucket_tree.py tests/test_gpu_sliced.py tests/test_gpu_config4.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/mar32 -o mar32 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 2 --reps 3 > $O/mar32.jsonl 2> $O/mar32.err || { tail -20 $O/mar32.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/mar64 -o mar64 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 1 --reps 3 > $O/mar64.jsonl 2> $O/mar64.err || { tail -20 $O/mar64.err; exit 1; }
cd $R
grep -o '"wall_ms": [0-9.]*\|"abs_err": [0-9.e-]*' $O/mar32.jsonl | tr '\n' ' '; echo
grep -o '"wall_ms": [0-9.]*\|"abs_err": [0-9.e-]*' $O/mar64.jsonl | tr '\n' ' '; echo
head -5 $(find $O/mar32 -name "*kernel_stats.csv") | cut -c1-150
head -5 $(find $O/mar64 -name "*kernel_stats.csv") | cut -c1-150
echo ok
