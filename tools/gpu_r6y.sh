# Sliced GPU tests (gloo worlds of 2 and 4 on the box's GPU: shares, relaunch).
set -o pipefail
R=$PWD
O=$R/gpurun_out/r6y; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sliced.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -12 $O/tests.log
