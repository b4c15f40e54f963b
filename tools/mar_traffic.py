#!/usr/bin/env python3
"""HBM traffic of the 32x32 MAR's split runs from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE) over tools/mar_grid.py: per kernel name, the launches
grouped by bytes read (gfx950 correction as tools/pmc_traffic.py: read bytes =
2 * FETCH_SIZE * 1024, written = WRITE_SIZE * 1024), to set beside the
algorithmic bytes (2^32 fp32 entries = 17.18 GB per message: an unfused run
reads one message and writes one; a run with a fused belief, kChainBel, also
reads the forward message and writes the 2^24-entry belief).

    python tools/mar_traffic.py FETCH.csv WRITE.csv > profiles/r04_mar32_traffic.json
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    out = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and ("chain_split_kernel<8" in r["Kernel_Name"] or
                                             "chain_split_kernel<float, 8" in r["Kernel_Name"] or
                                             "chain_split_kernel<double, " in r["Kernel_Name"]):
            out[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]) * 1024)
    return out


def main():
    fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
    res = {"correction": "read bytes = 2 * FETCH_SIZE * 1024 (gfx950, MI355X_MICROARCH.md HBM), "
                         "written = WRITE_SIZE * 1024; separate --pmc passes", "message_GB": {"f32": 2 ** 32 * 4 / 1e9, "f64": 2 ** 32 * 8 / 1e9},
           "kernels": {}}
    for k in sorted(fetch):
        groups = defaultdict(list)
        for i, fb in enumerate(fetch[k]):
            wb = write[k][i] if i < len(write.get(k, [])) else float("nan")
            msg = 34.36 if "<double" in k else 17.18         # GB per 2^32-entry message
            groups[round(2 * fb / 1e9 / msg)].append((2 * fb / 1e9, wb / 1e9))
        res["kernels"][k] = {
            "%d messages read" % g: {"launches": len(v), "read_GB": sum(a for a, _ in v) / len(v),
                                    "written_GB": sum(b for _, b in v) / len(v)}
            for g, v in sorted(groups.items())}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
