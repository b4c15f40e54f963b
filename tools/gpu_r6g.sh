# Round-6 evidence after the arena placement / kept-set changes: GPU suite,
# conditioned-PR and MAR kernel stats (fp32, fp64), split-run HBM traffic
# (separate FETCH_SIZE / WRITE_SIZE passes), then the bench line.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r6g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cond -o cond --output-format csv -- python3 $R/tools/cond_pr32.py --targets 0 --reps 2 > $O/cond.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/mar64 -o mar64 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 1 --reps 2 > $O/mar64.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/mar32 -o mar32 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 1 --reps 2 > $O/mar32.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/f64fetch -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 0 --reps 1 > $O/f64fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/f64write -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --check 0 --reps 1 > $O/f64write.log 2>&1 || exit 1
cd $R
python3 tools/mar_traffic.py $(find $O/f64fetch -name "*counter_collection.csv") $(find $O/f64write -name "*counter_collection.csv") > $O/mar64_traffic.json || exit 1
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo ok
