# Kernel trace of rank 0's share of the 8-rank sliced 32x32 MAR with the
# modelled xGMI time (delay kernels hold each exchange's stream): where the
# GPU idles while both lanes wait on exchanges.
set -o pipefail
R=$PWD
O=$R/gpurun_out/${R6V_OUT:-r6v}; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/sliced -o sliced --output-format csv -- python3 $R/tools/mar_sliced.py --ranks 8 --lanes 2 --reps 2 > $O/sliced.jsonl 2> $O/sliced.err || { tail -20 $O/sliced.err; exit 1; }
cd $R
cat $O/sliced.jsonl | cut -c1-300
echo ok
