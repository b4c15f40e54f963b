set -o pipefail
R=$PWD
O=$R/gpurun_out/r6m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sliced.py tests/test_gpu_bucket_tree.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 -u tools/mar_sliced.py --ranks 4 8 > $O/sliced.jsonl 2> $O/sliced.err || { tail -20 $O/sliced.err; exit 1; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/sl8 -o sl8 --output-format csv -- python3 $R/tools/mar_sliced.py --ranks 8 --reps 1 > $O/sl8.log 2>&1 || exit 1
echo ok
