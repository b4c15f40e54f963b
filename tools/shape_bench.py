#!/usr/bin/env python3
"""Per-shape kernel rates of the fused bucket (C ABI single-op path, HIP events
on one stream): the shapes that dominate the 32x32 bucket tree and the bench.

  fwd   forward message of a column sweep: m(y, S_1..S_n) * f(y, z) -> sum_y,
        output (S, z), z fastest (stream Col class)
  pi    backward message: m(S_1..S_n, y) * f(S_n, y) * u(y) -> sum_y, y the
        big input's fastest dim (stream interleaved class)
  col4  the bench bucket, k = 4, w = 14

    python tools/shape_bench.py [--n 28] [--reps 10]
"""
import argparse
import json
import os
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=28, help="binary S variables of fwd/pi (2^(n+1) big entries)")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import torch
    import bnpp

    ctx = bnpp.Context(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    n = args.n

    def rand(size):
        return torch.rand(size, generator=g, device=dev, dtype=torch.float32) * 1.5 + 0.5

    shapes = {}
    # fwd: vars 0 = y, 1..n = S, n+1 = z
    shapes["fwd"] = ([2] * (n + 2), [list(range(n + 1)), [0, n + 1]], 0)
    # pi: vars 0..n-1 = S, n = y
    shapes["pi"] = ([2] * (n + 1), [list(range(n + 1)), [n - 1, n], [n]], n)
    # pi2: the tree's backward message as planned: the parent variable xq (0) is
    # the output's slowest dim and absent from the big input (1..n = S, n+1 = y)
    shapes["pi2"] = ([2] * (n + 2), [list(range(1, n + 2)), [0, n + 1], [0]], n + 1)
    # col4: 0 = x, 1..14 = S, 15 = y
    shapes["col4"] = ([4] * 16, [list(range(15)), [0, 15]], 0)
    for name, (cards, scopes, elim) in shapes.items():
        if args.only and args.only != name:
            continue
        tabs = []
        for sc in scopes:
            size = 1
            for v in sc:
                size *= cards[v]
            tabs.append(rand(size))
        out_vars = bnpp.out_scope(scopes, elim)
        if name == "pi2":
            out_vars = [0] + list(range(1, n + 1))
        osz = 1
        for v in out_vars:
            osz *= cards[v]
        out = torch.empty(osz, device=dev, dtype=torch.float32)

        def step():
            bnpp.bucket_eliminate(ctx, bnpp.F32, cards, [t.data_ptr() for t in tabs], scopes, elim, out.data_ptr(),
                                  out_vars, stream=stream.cuda_stream)

        step()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        for a, b in ev:
            a.record(stream)
            step()
            b.record(stream)
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in ev)[len(ev) // 2]
        alg = 4 * (sum(t.numel() for t in tabs) + osz)
        print(json.dumps({"shape": name, "ms": ms, "alg_GB": alg / 1e9, "GBps": alg / ms / 1e6}), flush=True)
        del tabs, out
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
