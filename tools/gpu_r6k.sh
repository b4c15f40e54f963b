# Round-6 bench evidence (bench kernel trace + stats, FETCH_SIZE / WRITE_SIZE
# passes -> profiles/traffic_r06.json), and the N-GPU MAR projections on one
# GPU with the round-6 planner: message-sliced shares (loopback collective,
# xGMI time modelled) and the segment scheme's parts.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r6k; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="--no-cpu --no-mar --no-fp64"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 $B > $O/trace.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $B > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $B > $O/write.log 2>&1 || exit 1
cd $R
python3 tools/pmc_traffic.py $(find $O/fetch -name "*counter_collection.csv") $(find $O/write -name "*counter_collection.csv") --k 4 --w 14 > $O/traffic.json || exit 1
cat $O/traffic.json | head -30
timeout -k 10 600 python3 -u tools/mar_sliced.py --ranks 4 8 --one-rank > $O/sliced.jsonl 2> $O/sliced.err || { tail -20 $O/sliced.err; exit 1; }
timeout -k 10 600 python3 -u tools/mar_parts.py --parts 2 4 8 > $O/parts.jsonl 2> $O/parts.err || { tail -20 $O/parts.err; exit 1; }
echo ok
