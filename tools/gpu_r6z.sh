#!/bin/bash
# Sliced 32x32 MAR, 8-rank share on one GPU: the lanes' windows alternating
# (lane_order.hpp, BNPP_LANE_ALT = 1 strict, 0.5 half, 0 free-running as in
# round 6 before), tuning build lib_knobs, alternated; then the sliced GPU
# tests (alternating, tuning build) and the closing suite / smoke / bench on
# the product build.
set -o pipefail
R=$PWD
O=$R/gpurun_out/${R6Z_OUT:-r6z}; mkdir -p $O
export TMPDIR=/tmp
BNPP_LIB=$R/bn-pp_amd/lib_knobs/libbnpp.so BNPP_LANE_ALT=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_sliced.py > $O/sliced_tests.log 2>&1 || { tail -30 $O/sliced_tests.log; exit 1; }
tail -1 $O/sliced_tests.log
i=0
for a in 0 1 0.5 0 1; do
  i=$((i+1))
  BNPP_LIB=$R/bn-pp_amd/lib_knobs/libbnpp.so BNPP_LANE_ALT=$a timeout -k 10 300 python3 -u tools/mar_sliced.py --ranks 8 4 --lanes 2 --reps 3 > $O/alt_${i}_$a.jsonl 2> $O/alt_${i}_$a.err || { tail -20 $O/alt_${i}_$a.err; exit 1; }
  python3 -c "
import json
for l in open('$O/alt_${i}_$a.jsonl'):
    d = json.loads(l)
    print('alt $a ranks', d['ranks'], 'nocopy', [round(x, 1) for x in d['nocopy_walls_ms']], 'model_64', [round(x, 1) for x in d['model_64_walls_ms']])"
done
FINAL_OUT=${R6Z_OUT:-r6z}_final bash tools/gpu_final_r06a.sh
