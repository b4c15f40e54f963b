#!/usr/bin/env python3
"""Rate of the marginal-reduction bucket of the 32x32 bucket tree in isolation:
out[s] = sum_v a[v, s] * b[v, s] over a composite summed variable v (card 2048)
and s (card 2^21), two 2^32-entry fp32 inputs, through the single-op C ABI.

    python tools/red_bench.py [--reps 5]
"""
import argparse
import json
import os
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kv", type=int, default=2048)
    ap.add_argument("--ns", type=int, default=1 << 21)
    args = ap.parse_args()
    import torch
    import bnpp
    ctx = bnpp.Context(0)
    kv, ns = args.kv, args.ns
    dev = torch.device("cuda", 0)
    a = torch.rand(kv * ns, device=dev, dtype=torch.float32) + 0.5
    b = torch.rand(kv * ns, device=dev, dtype=torch.float32) + 0.5
    out = torch.empty(ns, device=dev, dtype=torch.float32)
    cards = [kv, ns]
    st = torch.cuda.Stream(dev)
    run = lambda: bnpp.bucket_eliminate(ctx, bnpp.F32, cards, [a.data_ptr(), b.data_ptr()], [[0, 1], [0, 1]], 0,
                                        out.data_ptr(), [1], stream=st.cuda_stream)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(args.reps):
        run()
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    want = (a.double().reshape(kv, ns) * b.double().reshape(kv, ns)).sum(0)
    err = ((out.double() - want).abs() / want).max().item()
    gb = 4.0 * (2 * kv * ns + ns) / 1e9
    print(json.dumps({"shape": "reduce %d x %d, 2 inputs" % (kv, ns), "ms": ms, "alg_GB": gb, "GBps": gb / ms * 1e3,
                      "max_rel_err": err}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
