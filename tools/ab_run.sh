set -o pipefail
bash tools/ab_libs.sh base mw6 mw8 base mw6 mw8 > gpurun_out/ab4.txt 2>&1
