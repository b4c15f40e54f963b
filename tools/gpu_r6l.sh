set -o pipefail
R=$PWD
O=$R/gpurun_out/r6l; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/sl8 -o sl8 --output-format csv -- python3 $R/tools/mar_sliced.py --ranks 8 --reps 1 > $O/sl8.log 2>&1 || exit 1
echo ok
