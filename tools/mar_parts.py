#!/usr/bin/env python3
"""Per-part cost of the sharded 32x32 bucket-tree MAR, measured on ONE GPU:
part r of N (bnpp_marginals_tree_part, what rank r runs under bench.py
--gpus N) timed warm, one part after the other.  The N-GPU wall-clock is the
slowest part plus one all-reduce of sum(card) fp64 values (16 KiB), so
max(part_ms) projects it without an N-GPU node.

    python tools/mar_parts.py --parts 2 4 8 > gpurun_out/mar_parts.jsonl
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32)
    ap.add_argument("--cols", type=int, default=32)
    ap.add_argument("--parts", type=int, nargs="+", default=[2, 4, 8])
    args = ap.parse_args()
    import bnpp
    from bnpp import synth
    r, c = args.rows, args.cols
    m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=0))
    col = [rr * c + cc for cc in range(c) for rr in range(r)]
    ctx = bnpp.Context(0)
    whole, _ = bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F32, order=col)
    for n in args.parts:
        ms, got = [], {}
        for p in range(n):
            bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F32, order=col, part=p, n_parts=n)     # warm
            t0 = time.perf_counter()
            mine, _ = bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F32, order=col, part=p, n_parts=n)
            ms.append((time.perf_counter() - t0) * 1e3)
            got.update(mine)
        err = max(abs(a - b) for t in whole for a, b in zip(whole[t], got[t]))
        print(json.dumps({"instance": "ising%dx%d-col" % (r, c), "dtype": "f32", "n_parts": n, "part_ms": ms,
                          "projected_wall_ms": max(ms), "owned_vars": len(got), "max_abs_diff_vs_whole": err}),
              flush=True)


if __name__ == "__main__":
    main()
