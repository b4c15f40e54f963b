set -o pipefail
O=gpurun_out/r6c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u tools/cond_pr32.py > $O/cond.jsonl 2> $O/cond.err || { tail -20 $O/cond.err; exit 1; }
cat $O/cond.jsonl
BNPP_TIMING=1 timeout -k 10 300 python3 -u tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 > $O/mar32.jsonl 2> $O/mar32.err || { tail -20 $O/mar32.err; exit 1; }
BNPP_TIMING=1 timeout -k 10 300 python3 -u tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 1 --reps 2 > $O/mar64.jsonl 2> $O/mar64.err || { tail -20 $O/mar64.err; exit 1; }
grep -E '"phase": "(mar|check)"' $O/mar32.jsonl $O/mar64.jsonl | cut -c1-220
echo ok
