#!/usr/bin/env python3
"""HBM traffic of the 32x32 MAR's largest slab / stream level launches (the
sweep's edge buckets) from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE; gfx950 correction as tools/mar_traffic.py), beside their
algorithmic bytes: the largest k=1 slab bucket [2^30][2][2] reads its 2^31-
entry big input twice (17.18 GB) and writes 2^32 entries (17.18 GB).

    python tools/edge_traffic.py FETCH.csv WRITE.csv > profiles/r04_mar32_edge_traffic.json
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    out = defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if r["Counter_Name"] == counter and ("slab_level_kernel" in n or "stream_level_kernel" in n):
            out[n.split("(")[0].replace("void bnpp::", "")].append(float(r["Counter_Value"]) * 1024)
    return out


def main():
    fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
    res = {"correction": "read bytes = 2 * FETCH_SIZE * 1024 (gfx950), written = WRITE_SIZE * 1024; separate --pmc passes",
           "kernels": {}}
    for k in sorted(fetch):
        pairs = [(2 * f / 1e9, (write[k][i] if i < len(write.get(k, [])) else float("nan")) / 1e9)
                 for i, f in enumerate(fetch[k])]
        pairs.sort(reverse=True)
        res["kernels"][k] = {"launches": len(pairs), "largest_read_written_GB": [[round(a, 3), round(b, 3)] for a, b in pairs[:4]]}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
