set -o pipefail
O=gpurun_out/r6b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u tools/cond_pr32.py > $O/cond.jsonl 2> $O/cond.err || { tail -20 $O/cond.err; exit 1; }
cat $O/cond.jsonl
R=$PWD; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o cond --output-format csv -- python3 $R/tools/cond_pr32.py --targets 0 --reps 2 --dtypes f32,f64 > $R/$O/prof.log 2>&1 || exit 1
echo ok
