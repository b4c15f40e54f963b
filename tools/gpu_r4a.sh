#!/bin/bash
# Round 4: cold-mapping probe + the new parity tests (partition sums, peaked
# potentials through the per-bucket fold).  Run on the GPU box from the repo root.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/r4a
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  "tests/test_gpu_bucket_tree.py::test_split_runs_peaked_potentials" \
  "tests/test_gpu_bucket_tree.py::test_split_runs_identical_to_unfused" tests/test_gpu_dist.py \
  tests/test_cpp_mirror.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 $R/tools/map_probe 240 > $OUT/map_probe.log 2>&1 || exit 1
BNPP_TIMING=1 timeout -k 10 200 python3 -u $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 2 > $OUT/mar.log 2>&1 || exit 1
timeout -k 10 120 python3 -u $R/tools/slab_ab.py > $OUT/slab_ab.jsonl 2> $OUT/slab_ab.err || exit 1
BNPP_TIMING=1 timeout -k 10 120 python3 -u $R/tools/pr_phases.py Mildew.uai Barley.uai pathfinder.uai Munin1.uai noisyor_50_80.uai:noisyor_50_80.uai.evid > $OUT/pr_phases.jsonl 2> $OUT/pr_phases.err || exit 1
timeout -k 10 200 python3 -u $R/tools/config4_bench.py > $OUT/config4_bench.jsonl 2> $OUT/config4_bench.err || exit 1
