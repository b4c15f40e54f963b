# Round-6 re-entry check on a rebuilt tree: GPU suite, smoke, bench (as the
# driver runs them), then a kernel trace of rank 0's share of the 8-rank sliced
# 32x32 MAR (compute alone) to break its 400 ms down by kernel and idle gaps.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r6s; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/sliced -o sliced --output-format csv -- python3 $R/tools/mar_sliced.py --ranks 8 --lanes 2 --no-model --reps 2 > $O/sliced.jsonl 2> $O/sliced.err || { tail -20 $O/sliced.err; exit 1; }
cd $R
cat $O/sliced.jsonl
echo ok
