#!/usr/bin/env python3
"""A/B of the slab bucket's tile shape on the bench bucket m(x, S_1..S_w) *
f(x, y) -> sum_x, f32 and f64, in one process -- BNPP_SLAB_V (slow-dim
entries per tile) and BNPP_SLAB_LANES=1 (one lane per 32-B tile row instead
of two):
kernel time from HIP events on the launch stream, best of --rounds rounds of
--steps launches, alternating the variants so box drift hits them alike.

    python tools/slab_ab.py > gpurun_out/slab_ab.jsonl
"""
import json
import os
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))


def main():
    import torch
    import bnpp
    k, w, steps, rounds = 4, 14, 10, 3
    dev = torch.device("cuda", 0)
    ctx = bnpp.Context(0)
    stream = torch.cuda.Stream(dev)
    S = k ** w
    cards = [k] * (w + 2)
    res = {}
    for dt, tdt, eb in ((bnpp.F32, torch.float32, 4), (bnpp.F64, torch.float64, 8)):
        g = torch.Generator(device=dev).manual_seed(1)
        m_t = torch.rand(k * S, generator=g, device=dev, dtype=tdt) + 0.5
        f_t = torch.rand(k * k, generator=g, device=dev, dtype=tdt) + 0.5
        outs = {}
        for r in range(rounds):
            for v in ("1:2", "1:1", "2:2", "2:1"):
                os.environ["BNPP_SLAB_V"], os.environ["BNPP_SLAB_LANES"] = v.split(":")
                out = torch.empty(S * k, device=dev, dtype=tdt)

                def step():
                    bnpp.bucket_eliminate(ctx, dt, cards, [m_t.data_ptr(), f_t.data_ptr()],
                                          [list(range(w + 1)), [0, w + 1]], 0, out.data_ptr(), list(range(1, w + 2)),
                                          stream=stream.cuda_stream)
                for _ in range(3):
                    step()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
                for i in range(steps):
                    ev[i][0].record(stream)
                    step()
                    ev[i][1].record(stream)
                torch.cuda.synchronize(dev)
                ms = sum(a.elapsed_time(b) for a, b in ev) / steps
                key = ("f32" if dt == bnpp.F32 else "f64", v)
                res[key] = min(res.get(key, 1e9), ms)
                if v in outs:
                    assert torch.equal(outs[v], out)
                outs[v] = out
        for v in outs:
            assert torch.equal(outs["1:2"], outs[v])          # same bits whatever the tile shape
        del m_t, f_t, outs
        torch.cuda.empty_cache()
    os.environ.pop("BNPP_SLAB_V", None)
    os.environ.pop("BNPP_SLAB_LANES", None)
    for (d, v), ms in sorted(res.items()):
        eb = 4 if d == "f32" else 8
        alg = eb * (2 * k * S + k * k)
        print(json.dumps({"dtype": d, "slab_v": int(v[0]), "lanes_per_32B_row": int(v[2]),
                          "kernel_ms": ms, "GBps": alg / ms / 1e6,
                          "frac": alg / ms / 1e6 / 8000.0}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
