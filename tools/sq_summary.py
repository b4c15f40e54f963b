#!/usr/bin/env python3
"""SQ counters of the 32x32 MAR's split runs from rocprofv3 --pmc passes over
tools/mar_grid.py (tools/final_sq_r04.sh): per kernel, per-dispatch averages
and per-wave instruction counts.  Backward runs with a fused belief
(kChainBel) are told apart from the others by their instruction counts (more
LDS and VMEM instructions per dispatch): a split at the midpoint of each
counter's range.

    python tools/sq_summary.py P1.csv P2.csv > profiles/r04_mar32_pmc_sq_final.json
"""
import csv
import json
import sys
from collections import defaultdict


def load(path):
    per = defaultdict(lambda: defaultdict(dict))       # kernel -> dispatch -> counter -> value
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void bnpp::", "")
        if "chain_split_kernel<8" not in k:
            continue
        per[k][r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    return per


def groups(disp, key):
    vals = [d.get(key, 0.0) for d in disp.values()]
    lo, hi = min(vals), max(vals)
    if hi <= lo * 1.2:
        return {"all": list(disp.values())}
    mid = (lo + hi) / 2
    return {"plain": [d for d in disp.values() if d.get(key, 0.0) < mid],
            "with belief": [d for d in disp.values() if d.get(key, 0.0) >= mid]}


def main():
    out = {"source": "tools/final_sq_r04.sh: rocprofv3 --pmc, two passes of SQ counters over one 32x32 MAR call "
                     "(tools/mar_grid.py); per-dispatch averages, and per wave = / SQ_WAVES", "kernels": {}}
    for path, key in ((sys.argv[1], "SQ_INSTS_LDS"), (sys.argv[2], "SQ_INSTS_VMEM_RD")):
        for k, disp in load(path).items():
            for g, ds in groups(disp, key).items():
                ent = out["kernels"].setdefault(k, {}).setdefault(g, {"per_dispatch": {}, "per_wave": {}})
                ent["dispatches_" + key] = len(ds)
                for c in sorted({c for d in ds for c in d}):
                    avg = sum(d.get(c, 0.0) for d in ds) / len(ds)
                    ent["per_dispatch"][c] = avg
                waves = ent["per_dispatch"].get("SQ_WAVES")
                if waves:
                    for c, v in ent["per_dispatch"].items():
                        if c.startswith("SQ_INSTS"):
                            ent["per_wave"][c] = v / waves
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
