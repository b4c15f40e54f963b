# Round-6 checkpoint: GPU suite, smoke, bench (as the driver runs them), and
# the arena's base address (BNPP_TIMING) for the placement notes.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r6q; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
BNPP_TIMING=1 timeout -k 10 300 python3 -u tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 0 --reps 1 > $O/mar64.jsonl 2> $O/mar64.err || exit 1
grep "arena" $O/mar64.err | grep "at 0x" | head -3
echo ok
