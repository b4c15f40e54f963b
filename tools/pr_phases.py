#!/usr/bin/env python3
"""Phase split of the GPU PR on the reference's large-card networks (the
MFMA question): host ordering + planning, upload, launch,
device run + fetch (bnpp_last_timing), median of --reps warm calls, beside
the bucket shapes (tools/bucket_shapes.py).  Run under rocprofv3
--kernel-trace --stats to get the kernel time of the same calls.

    python tools/pr_phases.py Mildew.uai Barley.uai pathfinder.uai > gpurun_out/pr_phases.jsonl
"""
import json
import os
import statistics
import sys
import time

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import bnpp  # noqa: E402
from bucket_shapes import MODELS, shapes  # noqa: E402


def main():
    reps = 5
    ctx = bnpp.Context(0)
    for a in sys.argv[1:]:
        name, _, evn = a.partition(":")
        m = bnpp.Model.load(os.path.join(MODELS, name))
        ev = bnpp.load_evidence(os.path.join(MODELS, evn)) if evn else {}
        bnpp.partition(ctx, m, ev, "mf", bnpp.F64)                     # cold
        walls, phases = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            lz, _, up = bnpp.partition(ctx, m, ev, "mf", bnpp.F64)
            walls.append((time.perf_counter() - t0) * 1e3)
            phases.append(bnpp.last_timing())
        med = {k: statistics.median(p[k] for p in phases) for k in phases[0]}
        sh = shapes(name, evn or None)
        print(json.dumps({"model": name, "evidence": evn or None, "log10Z": lz, "wall_ms_median": statistics.median(walls),
                          "phases_ms_median": med, "width": sh["width"], "factor_entries": sh["factor_entries"],
                          "largest_bucket": sh["top5"][0], "gemm_shaped_buckets": sh["gemm_shaped"]}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
