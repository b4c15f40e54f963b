# rocprofv3 evidence for bench.py (run on the GPU box from the repo root):
#   kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes.
set -e
R=$PWD
OUT=$R/gpurun_out/prof
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-mar > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-mar > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-mar > $OUT/write.log 2>&1
cd $R
timeout -k 10 300 python3 bench.py > $OUT/bench.log 2>&1
