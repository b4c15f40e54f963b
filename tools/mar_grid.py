#!/usr/bin/env python3
"""All marginals of an R x C Ising grid through the bucket tree (column-sweep
order), with a consistency check against conditioned partitions:
P(x_t = s) = Z(x_t = s) / Z  for a few targets t.

    python tools/mar_grid.py --rows 32 --cols 32 --check 2 > gpurun_out/mar32.jsonl
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
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--check", type=int, default=1, help="targets checked against conditioned partitions")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--reps", type=int, default=1, help="MAR calls on the same context (later ones warm)")
    args = ap.parse_args()
    import bnpp
    from bnpp import synth
    r, c = args.rows, args.cols
    dt = bnpp.F32 if args.dtype == "f32" else bnpp.F64
    import torch                                           # initialise torch's HIP runtime first
    free, _ = torch.cuda.mem_get_info(0)
    ctx = bnpp.Context(0)
    m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=args.seed))
    col = [rr * c + cc for cc in range(c) for rr in range(r)]
    if "BNPP_MEM_BUDGET_GB" not in os.environ:             # host-only stats: size them like the device run
        os.environ["BNPP_MEM_BUDGET_GB"] = str(free * 0.85 / 1e9)
        st = bnpp.plan_stats(m, 3, {}, "mf", dtype=dt, order=col)
        del os.environ["BNPP_MEM_BUDGET_GB"]
    else:
        st = bnpp.plan_stats(m, 3, {}, "mf", dtype=dt, order=col)
    pr_st = bnpp.plan_stats(m, 0, {}, "mf", dtype=dt, order=col)
    print(json.dumps({"phase": "plan", "tree_entries": st[0], "pr_entries": pr_st[0], "arena_GB": st[1] / 1e9,
                      "buckets": st[3], "alg_GB": st[6] / 1e9, "width": st[4]}), flush=True)
    for rep in range(args.reps):
        t0 = time.perf_counter()
        marg, up = bnpp.marginals_tree(ctx, m, {}, "mf", dt, order=col)
        wall = (time.perf_counter() - t0) * 1e3
        worst = max(abs(sum(p) - 1.0) for p in marg.values())
        print(json.dumps({"phase": "mar", "rep": rep, "instance": "ising%dx%d-col" % (r, c), "dtype": args.dtype,
                          "uptime_ms": up, "wall_ms": wall, "max_sum_err": worst,
                          "phases": bnpp.last_timing(),
                          "p0": marg[0], "p_mid": marg[(r // 2) * c + c // 2]}), flush=True)
    if args.check > 0:
        lz = bnpp.partition(ctx, m, {}, "mf", dt, order=col)[0]
        checks = [0, (r // 2) * c + c // 2, r * c - 1][: args.check]
        for t in checks:
            lz0 = bnpp.partition(ctx, m, {t: 0}, "mf", dt, order=col)[0]
            p0 = 10 ** (lz0 - lz)
            print(json.dumps({"phase": "check", "target": t, "mar": marg[t][0], "ratio_Z": p0,
                              "abs_err": abs(p0 - marg[t][0])}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
