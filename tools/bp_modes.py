#!/usr/bin/env python3
"""Loopy BP: the one-workgroup loop against the multi-workgroup flood
(BNPP_BP_MODE=single|multi) on the reference's networks and synthetic grids,
with the work estimate the automatic choice uses (capi.cpp kBpMultiWork).

    python tools/bp_modes.py > gpurun_out/bp_modes.jsonl
"""
import collections
import json
import os
import statistics
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))
import bnpp  # noqa: E402
from bnpp import synth  # noqa: E402

MODELS = os.path.join(REPO, "tests", "golden", "models")


def work(cards, scopes):
    w, deg = 0, collections.Counter()
    for s in scopes:
        size = 1
        for v in s:
            size *= cards[v]
            deg[v] += 1
        w += size * len(s) ** 2
    return w + sum(d * d * cards[v] for v, d in deg.items())


def cases():
    for name, eps in [("alarm.uai", 1e-3), ("andes.uai", 1e-3), ("Water.uai", 1e-3), ("pathfinder.uai", 1e-3),
                      ("Munin1.uai", 1e-3), ("Diabetes.uai", 1e-3), ("Link.uai", 1e-3), ("ising12x12.uai", 1e-6)]:
        p = os.path.join(MODELS, name)
        if os.path.exists(p):
            yield name, bnpp.Model.load(p), synth.read_uai(p), eps
    for n in (32, 64, 128, 256):
        d = synth.ising_grid(n, n, seed=5)
        yield "ising%dx%d" % (n, n), bnpp.Model.from_dict(d), d, 1e-6
    d = synth.noisy_or_bn(200, 400, 6, seed=5)
    yield "noisyor200x400", bnpp.Model.from_dict(d), d, 1e-3


def main():
    ctx = bnpp.Context(0)
    for name, m, d, eps in cases():
        rec = {"instance": name, "eps": eps}
        if d is not None:
            rec["work"] = work(d["cards"], d["scopes"])
        for mode in ("single", "multi"):
            os.environ["BNPP_BP_MODE"] = mode
            bnpp.sum_product(ctx, m, 10000, eps)
            ts = []
            for _ in range(3):
                _, it, up = bnpp.sum_product(ctx, m, 10000, eps)
                ts.append(up)
            rec[mode + "_ms"] = statistics.median(ts)
            rec[mode + "_it"] = it
        os.environ.pop("BNPP_BP_MODE")
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
