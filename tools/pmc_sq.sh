#!/bin/bash
# SQ instruction-mix counters of the split chain runs: the engine on the
# 32x32 MAR (one call) against tools/splitbw.hip's replica of the same run.
# Two --pmc passes per program (<= 8 SQ counters each).  (GPU box, repo root)
set -o pipefail
R=$PWD
export TMPDIR=/tmp
OUT=$R/gpurun_out/pmc_sq
mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $P -d $OUT/mar$i -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 32 --check 0 --reps 1 > $OUT/mar$i.log 2>&1) || { tail -3 $OUT/mar$i.log; exit 1; }
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/mb$i -o k --output-format csv -- $R/build/splitbw > $OUT/mb$i.log 2>&1) || { tail -3 $OUT/mb$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, re, sys, collections
for sub in ("mar", "mb"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for i in (1, 2):
        f = glob.glob("%s/%s%d/**/*counter_collection.csv" % (sys.argv[1], sub, i), recursive=True)[0]
        for r in csv.DictReader(open(f)):
            k = re.sub(r'\(.*', '', r["Kernel_Name"])
            if not re.search(r"chain_split|fwd|bwd|copy", k): continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(k, r["Counter_Name"])] += 1
    for k, d in acc.items():
        waves = d["SQ_WAVES"] / max(1, n[(k, "SQ_WAVES")])
        per = {c.replace("SQ_", ""): d[c] / max(1, n[(k, c)]) for c in d}
        print(sub, k[:60], "dispatches", n[(k, "SQ_WAVES")] // 2,
              " ".join("%s=%.4g" % (c, v / waves if not c.endswith("CYCLES") and c != "WAVES" else v) for c, v in sorted(per.items())))
PY
