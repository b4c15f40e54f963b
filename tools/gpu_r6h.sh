# A/B of the passes per block of the 8-input slab class on the conditioned
# 32x32 PR's 5-input bucket (BNPP_SLAB_R in a -DBNPP_TUNING_KNOBS build), and
# the parity tests of the default build.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r6h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bucket_tree.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
for r in 1 2 4; do
  BNPP_LIB=$R/bn-pp_amd/lib_knobs/libbnpp.so BNPP_SLAB_R=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r$r -o cond --output-format csv -- python3 $R/tools/cond_pr32.py --targets 0 --reps 2 > $O/r$r.log 2>&1 || exit 1
  grep -h "slab_level_kernel<[a-z]*, 2, 4, 1, [12], [124], 8>" $(find $O/r$r -name "*kernel_stats.csv") | cut -d, -f1-6
  grep log10Z $O/r$r.log | cut -c1-90
done
echo ok
