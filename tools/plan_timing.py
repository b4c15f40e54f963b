#!/usr/bin/env python3
"""Host planning time of the 32x32 column-sweep bucket tree (bnpp_plan_stats,
no GPU); BNPP_TIMING=1 prints the phases.  Run on the GPU box for its CPU."""
import sys, time
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "..", "bn-pp_amd", "python"))
import bnpp
from bnpp import synth
r = c = 32
m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=1))
col = [i * c + j for j in range(c) for i in range(r)]
for rep in range(3):
    t = time.time()
    st = bnpp.plan_stats(m, 3, None, "mf", bnpp.F32, order=col)
    print("plan_stats kind 3: %.1f ms" % ((time.time() - t) * 1e3), st[:4], flush=True)
