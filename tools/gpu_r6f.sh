set -o pipefail
O=gpurun_out/r6f; mkdir -p $O
M="timeout -k 10 300 python3 -u tools/mar_grid.py --rows 32 --cols 32 --dtype f64 --reps 2"
$M --check 1 > $O/a_default.jsonl 2> $O/a.err || exit 1
BNPP_KEEP_LOG2=24 $M --check 1 > $O/b_keep24.jsonl 2> $O/b.err || exit 1
BNPP_LIB=bn-pp_amd/lib_bel8/libbnpp.so BNPP_KEEP_LOG2=24 $M --check 2 > $O/c_bel8_keep24.jsonl 2> $O/c.err || exit 1
grep -h -E '"phase": "(mar|check)"' $O/a_default.jsonl $O/b_keep24.jsonl $O/c_bel8_keep24.jsonl | cut -c1-160
echo ok
