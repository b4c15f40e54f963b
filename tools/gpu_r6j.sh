set -o pipefail
R=$PWD
O=$R/gpurun_out/r6j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
BNPP_TIMING=1 timeout -k 10 300 python3 -u tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 > $O/mar32.jsonl 2> $O/mar32.err || { tail -20 $O/mar32.err; exit 1; }
BNPP_TIMING=1 timeout -k 10 300 python3 -u tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 1 --reps 2 > $O/mar64.jsonl 2> $O/mar64.err || { tail -20 $O/mar64.err; exit 1; }
grep -h -E '"phase": "(mar|check)"' $O/mar32.jsonl $O/mar64.jsonl | cut -c1-140
grep -h "checkpoint slots\|arena" $O/mar32.err $O/mar64.err | sort | uniq -c | head
echo ok
