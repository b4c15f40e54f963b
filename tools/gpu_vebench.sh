# VE wall-clock table (tools/ve_bench.py --ref); a heartbeat file keeps the
# box's hang detector informed while the single-core reference runs
set -o pipefail
mkdir -p gpurun_out
(while true; do date > gpurun_out/heartbeat; sleep 50; done) &
HB=$!
timeout -k 10 1100 python -u tools/ve_bench.py --ref --ref-timeout 150 > gpurun_out/ve_bench.jsonl 2> gpurun_out/ve_bench.err
rc=$?
kill $HB
exit $rc
