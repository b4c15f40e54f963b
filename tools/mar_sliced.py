#!/usr/bin/env python3
"""Projection of the message-sliced 32x32 bucket-tree MAR on N
GPUs from one GPU: rank 0's share of bnpp_marginals_tree_sliced run with the
loopback collective, twice -- moving the exchanged bytes locally ("copy":
device-to-device) and moving none ("nocopy": the compute alone) -- plus the
exchange volume the plan states (bytes this rank sends per call).

Every rank of a sliced run executes the same schedule on a block of the same
size, so rank 0's time is the world's compute time.  The projected N-GPU
wall-clock = nocopy time + exchange bytes / (links x per-link bandwidth),
without overlap of exchanges and compute.  xGMI on MI355X: 7 links per GPU,
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
    ap.add_argument("--link-gbs", type=float, default=64.0)
    ap.add_argument("--one-rank", action="store_true", help="also time the one-rank tree (reference point)")
    args = ap.parse_args()
    r, c = args.rows, args.cols
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
        _, st = bnpp.plan_tree_sliced(m, 0, R, order=col)
        rec = {"instance": "ising%dx%d-col" % (r, c), "ranks": R, "entries_per_rank": st[0], "arena_GB": st[1] / 1e9,
               "buckets": st[3], "exchanges": st[8], "bytes_sent_per_rank_GB": st[9] / 1e9}
        for mode in ("nocopy", "copy"):
            ts = []
            for _ in range(args.reps):
                t = time.perf_counter()
                bnpp.marginals_tree_sliced(ctx, m, 0, R, "loopback-" + mode if mode == "nocopy" else "loopback",
                                           order=col)
                ts.append((time.perf_counter() - t) * 1e3)
            rec[mode + "_ms"] = min(ts)
            rec[mode + "_walls_ms"] = ts
        links = min(R - 1, 7)
        xfer = st[9] / (links * args.link_gbs * 1e9) * 1e3
        rec.update({"links_per_rank": links, "link_GBps_assumed": args.link_gbs, "xgmi_ms": xfer,
                    "projected_ms": rec["nocopy_ms"] + xfer,
                    "note": "projection: compute of one rank (every rank's share is the same size) + exchange "
                            "bytes over R-1 xGMI links, no overlap"})
        print(json.dumps(rec), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
