set -o pipefail
O=gpurun_out/r6a; mkdir -p $O
bash tools/nodefer_diag.sh > $O/diag.log 2>&1 || { echo diag failed; exit 1; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
BNPP_BENCH_REHEARSE=1 timeout -k 10 400 python3 -u bench.py --gpus 2 --no-mar-f64 --mar-rows 16 --mar-cols 16 --secondary ising10x10.uai > $O/rehearse2.json 2> $O/rehearse2.err || { tail -20 $O/rehearse2.err; exit 1; }
echo all ok
