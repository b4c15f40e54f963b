set -o pipefail
R=$PWD
O=$R/gpurun_out/r6e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 -u bench.py --no-mar-f64 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; b=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(b['value'], b['roofline']['frac'], b['fp64_bucket']['frac'], b['mar']['wall_ms'])"
echo ok
