#!/usr/bin/env python3
"""Loopy BP flood on one synthetic Ising grid, for a kernel trace:
    rocprofv3 --kernel-trace --stats -d gpurun_out/bpprof -o bp -- python3 tools/bp_prof.py 128
"""
import os
import sys
import time

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))
import bnpp  # noqa: E402
from bnpp import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
os.environ.setdefault("BNPP_BP_MODE", "multi")
ctx = bnpp.Context(0)
m = bnpp.Model.from_dict(synth.ising_grid(n, n, seed=5))
for _ in range(3):
    t = time.time()
    _, it, up = bnpp.sum_product(ctx, m, 10000, 1e-6)
    print("ising%d %s: %d iterations, %.2f ms (%.1f us per iteration)" % (n, os.environ["BNPP_BP_MODE"], it, up,
                                                                         1e3 * up / max(it, 1)), flush=True)
