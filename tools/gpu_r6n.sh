set -o pipefail
R=$PWD
O=$R/gpurun_out/r6n; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for r in 29 30; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/m$r -o m --output-format csv -- python3 $R/tools/mar_grid.py --rows $r --cols 32 --check 0 --reps 2 > $O/m$r.log 2>&1 || exit 1
done
echo ok
