#!/bin/bash
# Closing evidence with the lanes' windows alternating by default (product
# build): sliced GPU tests, the 8- and 4-rank sliced projection, the GPU suite,
# smoke, bench line and kernel trace (gpu_final_r06a.sh), and the self-launched
# two-rank bench rehearsal (sliced MAR over gloo on one GPU).
set -o pipefail
R=$PWD
O=$R/gpurun_out/r6zz; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_sliced.py > $O/sliced_tests.log 2>&1 || { tail -30 $O/sliced_tests.log; exit 1; }
tail -1 $O/sliced_tests.log
timeout -k 10 300 python3 -u tools/mar_sliced.py --ranks 8 4 --lanes 2 --reps 3 > $O/sliced.jsonl 2> $O/sliced.err || { tail -20 $O/sliced.err; exit 1; }
python3 -c "
import json
for l in open('$O/sliced.jsonl'):
    d = json.loads(l)
    print('ranks', d['ranks'], 'nocopy', [round(x, 1) for x in d['nocopy_walls_ms']], 'model_64', [round(x, 1) for x in d['model_64_walls_ms']])"
FINAL_OUT=r6zz_final bash tools/gpu_final_r06a.sh || exit 1
BNPP_BENCH_REHEARSE=1 timeout -k 10 500 python3 -u bench.py --gpus 2 --no-mar-f64 --mar-rows 16 --mar-cols 16 > $O/rehearse2.json 2> $O/rehearse2.err || { tail -20 $O/rehearse2.err; exit 1; }
python3 -c "
import json
d = json.loads(open('$O/rehearse2.json').read().strip().splitlines()[-1])
m = d['mar']
print('rehearse world', d['world_size'], 'ok', d['checksum_ok'], 'cpu', d['cpu_baseline'] is not None, 'mar scheme', m.get('scheme'), 'sliced ok', (m.get('sliced') or {}).get('ok', m.get('ok')))"
