#!/usr/bin/env python3
"""A/B of two builds of libbnpp.so (BNPP_LIB) on the buckets the generic
gather kernels run: the 32x32 column-sweep PR conditioned on x_0 (a 5-input
bucket over an 8-GiB message) in fp32 and fp64, and fp64 PR on every network
of tests/golden/models.  Warm medians of 3 calls after a cold one; run under
rocprofv3 --kernel-trace --stats for the kernels' own time.

    BNPP_LIB=build_ab/libbnpp_base.so python tools/generic_ab.py > gpurun_out/ab_base.jsonl
"""
import glob
import json
import os
import statistics
import sys
import time

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))
import bnpp  # noqa: E402
from bnpp import synth  # noqa: E402


def timed(fn, reps=3):
    out = fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return statistics.median(ts), out


def main():
    ctx = bnpp.Context(0)
    lib = os.path.basename(os.path.dirname(bnpp.LIB_PATH)) + "/" + os.path.basename(bnpp.LIB_PATH)
    r = c = 32
    m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=1))
    col = [i * c + j for j in range(c) for i in range(r)]
    for dt, name in ((bnpp.F32, "f32"), (bnpp.F64, "f64")):
        ms, (lz, _) = timed(lambda: bnpp.partition(ctx, m, {0: 0}, "mf", dt, order=col)[:2])
        print(json.dumps({"lib": lib, "case": "ising32x32 PR x0=0 " + name, "warm_ms": ms, "log10Z": lz}), flush=True)
    for path in sorted(glob.glob(os.path.join(REPO, "tests", "golden", "models", "*.uai"))):
        mm = bnpp.Model.load(path)
        try:
            ms, (lz, _) = timed(lambda: bnpp.partition(ctx, mm, {}, "mf", bnpp.F64)[:2])
        except bnpp.BnppError as e:
            print(json.dumps({"lib": lib, "case": os.path.basename(path), "error": str(e)}), flush=True)
            continue
        print(json.dumps({"lib": lib, "case": os.path.basename(path), "warm_ms": ms, "log10Z": lz}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
