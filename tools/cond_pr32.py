#!/usr/bin/env python3
"""The 32x32 column-sweep PR conditioned on x_t (the bench's MAR check): wall
per call, warm, fp32 and fp64, log10 Z printed so builds can be compared bit
for bit.  Under rocprofv3 --kernel-trace the 5-input bucket of the x_0 case
shows as its own kernel.

    python tools/cond_pr32.py [--targets 0,528] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))
import bnpp  # noqa: E402
from bnpp import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--targets", default="0,528")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--dtypes", default="f32,f64")
a = ap.parse_args()
ctx = bnpp.Context(0)
m = bnpp.Model.from_dict(synth.ising_grid(32, 32, seed=0))
order = [r * 32 + c for c in range(32) for r in range(32)]
for dn in a.dtypes.split(","):
    dt = bnpp.F32 if dn == "f32" else bnpp.F64
    for t in [int(x) for x in a.targets.split(",")]:
        ms = []
        for i in range(a.reps):
            t0 = time.perf_counter()
            lz = bnpp.partition(ctx, m, {t: 0}, "mf", dt, order=order)[0]
            ms.append((time.perf_counter() - t0) * 1e3)
        print(json.dumps({"dtype": dn, "target": t, "log10Z": repr(lz), "ms": ms, "warm_ms": min(ms[1:] or ms)}),
              flush=True)
ctx.close()
