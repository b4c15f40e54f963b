set -o pipefail
AB_VE=1 bash tools/ab_libs.sh base mwide base mwide > gpurun_out/ab6.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || exit 1
