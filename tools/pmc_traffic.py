#!/usr/bin/env python3
"""HBM bytes per launch of the bench kernel from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE; counter CSVs), with the gfx950 correction of
MI355X_MICROARCH.md (HBM): FETCH_SIZE reports half the bytes of wide coalesced
streaming reads, so bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv --k 4 --w 14 > profiles/traffic_r02.json
"""
import argparse
import csv
import json


def per_launch(path, counter, kernel_sub):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and kernel_sub in r["Kernel_Name"]]
    return sum(vals) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--w", type=int, default=14)
    ap.add_argument("--kernel", default="slab_single_kernel")
    ap.add_argument("--dtype", choices=["f32", "f64"], default="f32")
    args = ap.parse_args()
    f, nf = per_launch(args.fetch, "FETCH_SIZE", args.kernel)
    w, nw = per_launch(args.write, "WRITE_SIZE", args.kernel)
    names = {r["Kernel_Name"] for r in csv.DictReader(open(args.fetch)) if args.kernel in r["Kernel_Name"]}
    S = args.k ** args.w
    eb = 4 if args.dtype == "f32" else 8
    alg = eb * (args.k * S + args.k * args.k + S * args.k)
    print(json.dumps({
        "k": args.k, "w": args.w, "dtype": args.dtype, "kernel": sorted(names),
        "launches": [nf, nw],
        "FETCH_SIZE_KB_per_launch": f, "WRITE_SIZE_KB_per_launch": w,
        "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024,
        "correction": "gfx950: FETCH_SIZE reports half the bytes of wide coalesced streaming reads "
                      "(MI355X_MICROARCH.md, HBM); bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024; "
                      "separate --pmc passes for FETCH_SIZE and WRITE_SIZE",
        "algorithmic_bytes_per_launch": alg,
        "source": "tools/profile_bench.sh (rocprofv3 --pmc, one counter per pass)"}, indent=1))


if __name__ == "__main__":
    main()
