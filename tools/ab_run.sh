set -o pipefail
for g in 3 4; do echo "== grid $g" ; BNPP_GRID_PER_CU=$g AB_VE=1 bash tools/ab_libs.sh base ntl || exit 1; done > gpurun_out/ab2.txt 2>&1
