# rocprofv3 evidence (run on the GPU box from the repo root):
#   bench kernel trace + stats, FETCH_SIZE and WRITE_SIZE in separate PMC passes,
#   the 32x32 bucket-tree MAR kernel stats, then the full bench line.
set -e
R=$PWD
OUT=$R/gpurun_out/prof
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="--no-cpu --no-mar --no-fp64"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 $B > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $B > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $B > $OUT/write.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/mar32 -o mar32 --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 3 --reps 2 > $OUT/mar32.log 2>&1
cd $R
python3 tools/pmc_traffic.py $(find $OUT/fetch -name "*counter_collection.csv") $(find $OUT/write -name "*counter_collection.csv") > $OUT/traffic.json
timeout -k 10 600 python3 bench.py > $OUT/bench.log 2>&1
