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
