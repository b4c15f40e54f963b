set -o pipefail
bash tools/ab_libs.sh base x2 base x2 > gpurun_out/ab5.txt 2>&1
