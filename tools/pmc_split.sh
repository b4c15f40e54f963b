#!/bin/bash
# SQ counters of the chain kernels on the 32x32 MAR (one pass) and of the
# chainbw microbenchmark kernels, for the split-form investigation.
set -o pipefail
R=$PWD
export TMPDIR=/tmp
L=${LIB:-$R/bn-pp_amd/lib/libbnpp.so}
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
mkdir -p $R/gpurun_out/pmc_split
(cd /tmp && BNPP_LIB=$L timeout -s KILL 240 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_split/mar -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 1 > $R/gpurun_out/pmc_split/mar.log 2>&1) || exit 1
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_split/mb -o k --output-format csv -- $R/build/chainbw > $R/gpurun_out/pmc_split/mb.log 2>&1) || exit 1
python3 - $R/gpurun_out/pmc_split <<'PY'
import csv, glob, re, sys, collections
for sub in ("mar", "mb"):
    f = glob.glob(sys.argv[1] + "/" + sub + "/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = re.sub(r'\(.*', '', r["Kernel_Name"])
        if not re.search(r"chain|fwd|bwd|copy", k): continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
    for k, d in acc.items():
        calls = n[(k, "SQ_WAVES")]
        print(sub, k[:60], "calls", calls, " ".join("%s=%.3g" % (c.replace("SQ_", ""), v / max(calls, 1)) for c, v in sorted(d.items())))
PY
