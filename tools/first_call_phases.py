#!/usr/bin/env python3
"""Phase split of first calls on fresh models (config 4 and the 16x16 grid):
is a first call's excess over a relaunch per model (ordering, planning,
uploads, arena) or per process (kernel code objects loaded at first launch)?
Three fresh loads of the same file in a row; bnpp.last_timing() after each.

    BNPP_TIMING=1 python tools/first_call_phases.py > gpurun_out/first_calls.jsonl
"""
import json
import os
import sys
import time

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))
import bnpp  # noqa: E402

G = os.path.join(REPO, "tests", "golden")
ctx = bnpp.Context(0)
warm = bnpp.Model.load(os.path.join(G, "models", "asia.uai"))
for dt in (bnpp.F64, bnpp.F32):
    bnpp.partition(ctx, warm, {}, "mf", dt)
    bnpp.marginals_tree(ctx, warm, {}, "mf", dt)
with open(os.path.join(G, "config4_golden.json")) as f:
    g = json.load(f)
path = os.path.join(G, "models", g["model"])
ev = bnpp.load_evidence(os.path.join(G, "models", g["evidence"]))
for kind in ("pr", "tree"):
    for dt, name in ((bnpp.F64, "f64"), (bnpp.F32, "f32")):
        for i in range(3):
            m = bnpp.Model.load(path)
            t0 = time.perf_counter()
            if kind == "pr":
                bnpp.partition(ctx, m, ev, "mf", dt)
            else:
                bnpp.marginals_tree(ctx, m, ev, "mf", dt)
            ms = (time.perf_counter() - t0) * 1e3
            print(json.dumps({"kind": kind, "dtype": name, "load": i, "ms": ms, "phases": bnpp.last_timing()}),
                  flush=True)
ctx.close()
