#!/usr/bin/env python3
"""Projection of the message-sliced 32x32 bucket-tree MAR on N
GPUs from one GPU: rank 0's share of bnpp_marginals_tree_sliced run with the
loopback collective: moving no bytes ("nocopy": the compute alone), and with
every exchange's stream held for its modelled xGMI duration ("model": the
lanes' overlap of exchanges and buckets measured, the link time modelled),
with the two-lane schedule and with one lane (BNPP_SLICE_LANES=0), plus the
exchange volume the plan states (bytes this rank sends per call).

Every rank of a sliced run executes the same schedule on a block of the same
size, so rank 0's time is the world's compute time.  The projected N-GPU
wall-clock is the "model" time (serial bound: nocopy + exchange bytes /
(links x per-link bandwidth)).  xGMI on MI355X: 7 links per GPU,
153.6 GB/s per link both directions together (76.8 GB/s each way); an
all-to-all over R ranks uses R-1 links in each direction at once; --link-gbs
sets the achieved per-direction rate (default 64 GB/s, 83 % of 76.8).

    python tools/mar_sliced.py --ranks 2 4 8 > gpurun_out/mar_sliced.jsonl
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32)
    ap.add_argument("--cols", type=int, default=32)
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--link-gbs", type=float, nargs="+", default=[64.0])
    ap.add_argument("--latency-us", type=int, default=20, help="per collective (3 per exchange: sync, data)")
    ap.add_argument("--one-rank", action="store_true", help="also time the one-rank tree (reference point)")
    ap.add_argument("--lanes", type=int, nargs="+", default=[2, 1], help="schedules to time (2: two fronts, 1: one)")
    ap.add_argument("--no-model", action="store_true", help="time the compute alone (nocopy) only")
    args = ap.parse_args()
    r, c = args.rows, args.cols
    # the run and the plan statistics see the same budget (the plan-only call
    # has no device to ask); 0.85 x 288 GB, what a fresh MI355X reports
    os.environ.setdefault("BNPP_MEM_BUDGET_GB", "240")
    m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=0))
    col = [i * c + j for j in range(c) for i in range(r)]
    ctx = bnpp.Context(0)
    if args.one_rank:
        ts = []
        for _ in range(args.reps):
            t = time.perf_counter()
            bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F32, order=col)
            ts.append((time.perf_counter() - t) * 1e3)
        print(json.dumps({"instance": "ising%dx%d-col" % (r, c), "ranks": 1, "wall_ms": min(ts), "walls_ms": ts}),
              flush=True)
    for R in args.ranks:
        for nl in args.lanes:
            lanes = 1 if nl == 2 else 0
            os.environ["BNPP_SLICE_LANES"] = str(lanes)
            _, st = bnpp.plan_tree_sliced(m, 0, R, order=col)
            rec = {"instance": "ising%dx%d-col" % (r, c), "ranks": R, "lanes": 2 if lanes else 1,
                   "entries_per_rank": st[0], "arena_GB": st[1] / 1e9, "buckets": st[3], "exchanges": st[8],
                   "bytes_sent_per_rank_GB": st[9] / 1e9}
            modes = {"nocopy": "loopback-nocopy"}
            for g in ([] if args.no_model else args.link_gbs):
                modes["model_%g" % g] = "loopback-model:%d:%d" % (int(g * 1000), args.latency_us)
            for name, coll in modes.items():
                ts = []
                for _ in range(args.reps):
                    t = time.perf_counter()
                    bnpp.marginals_tree_sliced(ctx, m, 0, R, coll, order=col)
                    ts.append((time.perf_counter() - t) * 1e3)
                rec[name + "_ms"] = min(ts)
                rec[name + "_walls_ms"] = ts
            links = min(R - 1, 7)
            rec.update({"links_per_rank": links, "latency_us": args.latency_us})
            for g in ([] if args.no_model else args.link_gbs):
                xfer = st[9] / (links * g * 1e9) * 1e3 + st[8] * 3 * args.latency_us * 1e-3
                rec["xgmi_ms_%g" % g] = xfer
                rec["serial_projection_ms_%g" % g] = rec["nocopy_ms"] + xfer
            rec["note"] = ("model_<GB/s>_ms: measured on one GPU with every exchange's stream held for its modelled "
                           "xGMI time (latency + bytes over R-1 links at <GB/s> each way), so the lanes' overlap is "
                           "measured; serial_projection: compute + transfers back to back")
            print(json.dumps(rec), flush=True)
    os.environ.pop("BNPP_SLICE_LANES", None)
    ctx.close()


if __name__ == "__main__":
    main()
