# Sliced MAR with the backward lane's pack folded into its unpack (xchg mode 2):
# sliced GPU tests (gloo worlds on the box's GPU, one-rank RCCL), then rank 0's
# share of the 32x32 MAR at 4 and 8 ranks (compute alone and modelled xGMI).
set -o pipefail
R=$PWD
O=$R/gpurun_out/r6u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sliced.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 -u tools/mar_sliced.py --ranks 4 8 --lanes 2 --reps 2 > $O/sliced.jsonl 2> $O/sliced.err || { tail -20 $O/sliced.err; exit 1; }
python3 -c "
import json
for l in open('$O/sliced.jsonl'):
    d=json.loads(l); print(d['ranks'], 'nocopy %.1f model %.1f sent %.1f GB' % (d['nocopy_ms'], d['model_64_ms'], d['bytes_sent_per_rank_GB']))"
echo ok
