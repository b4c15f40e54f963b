set -o pipefail
R=$PWD
O=$R/gpurun_out/r6p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bucket_tree.py tests/test_gpu_sliced.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/mar32 -o mar32 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 > $O/mar32.log 2>&1 || exit 1
echo ok
