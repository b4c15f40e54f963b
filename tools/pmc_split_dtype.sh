#!/bin/bash
# SQ counters of the split chain runs, fp32 against fp64: one 32x4 grid MAR
# per dtype (tools/mar_grid.py), two --pmc passes each (<= 8 SQ counters).
# Per kernel: per-dispatch averages, and per wave (/ SQ_WAVES).  (GPU box)
set -o pipefail
R=$PWD
export TMPDIR=/tmp
OUT=$R/gpurun_out/pmc_dt
mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
for dt in f32 f64; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $P -d $OUT/${dt}_$i -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 4 --dtype $dt --check 0 --reps 1 > $OUT/${dt}_$i.log 2>&1) || { tail -5 $OUT/${dt}_$i.log; exit 1; }
  done
  (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/${dt}_kt -o k --output-format csv -- python3 $R/tools/mar_grid.py --rows 32 --cols 4 --dtype $dt --check 0 --reps 1 > $OUT/${dt}_kt.log 2>&1) || { tail -5 $OUT/${dt}_kt.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, re, sys, collections
out = sys.argv[1]
for dt in ("f32", "f64"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for i in (1, 2):
        f = glob.glob("%s/%s_%d/**/*counter_collection.csv" % (out, dt, i), recursive=True)[0]
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void bnpp::", "")
            if "chain_split" not in k: continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(k, r["Counter_Name"])] += 1
    for k, d in sorted(acc.items()):
        per = {c: d[c] / max(1, n[(k, c)]) for c in d}
        waves = per.get("SQ_WAVES", 1.0)
        wc = per.get("SQ_WAVE_CYCLES", 1.0)
        print(dt, k, "dispatches", n[(k, "SQ_WAVES")] // 2, "waves/disp %.0f" % waves)
        print("   cycles share: " + " ".join("%s=%.3f" % (c.replace("SQ_", ""), per[c] / wc) for c in
              ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS") if c in per))
        print("   per wave: " + " ".join("%s=%.0f" % (c.replace("SQ_INSTS_", ""), per[c] / waves) for c in sorted(per) if c.startswith("SQ_INSTS")))
        print("   BUSY_CYCLES=%.4g WAVE_CYCLES=%.4g" % (per.get("SQ_BUSY_CYCLES", 0), wc))
PY
for dt in f32 f64; do echo "== $dt"; head -8 $(find $OUT/${dt}_kt -name "*kernel_stats.csv") | cut -c1-200; done
