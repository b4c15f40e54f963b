set -o pipefail
R=$PWD
OUT=$R/gpurun_out/prof_mar32
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o mar32 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 > $OUT/mar32.log 2>&1
