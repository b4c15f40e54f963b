#!/usr/bin/env python3
"""VE wall-clock on grid instances: GPU engine vs the reference CPU path.

For each instance prints one JSON line with
  gpu_uptime_ms   first call of bnpp.partition / bnpp.marginals: ordering +
                  planning + upload + device run + fetch (the reference's
                  "Executed in" scope, model.cpp:258/296 and 309/341)
  gpu_launch_ms   steady-state device time of the prepared job (launch + fetch)
  ref_ms          reference CPU (oracle/_ref/ref_harness, one core) when
                  --ref is given and the instance is reference-runnable
Run on the GPU box:  python tools/ve_bench.py --ref > gpurun_out/ve_bench.jsonl
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))


def ref_time(kind, path, timeout, evid="-"):
    h = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    if not os.path.exists(h):
        return None
    try:
        out = subprocess.run(["taskset", "-c", "0", h, kind, path, evid, "mf"], capture_output=True, text=True,
                             timeout=timeout, check=True).stdout
    except subprocess.TimeoutExpired:
        return {"timeout_s": timeout}
    for line in out.splitlines():
        p = line.split()
        if len(p) == 2 and p[0] == "uptime_ms":
            return float(p[1])
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", action="store_true", help="also time the reference CPU path (single core)")
    ap.add_argument("--ref-timeout", type=float, default=120)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import bnpp
    from bnpp import synth

    ctx = bnpp.Context(0)
    cases = [("ising10x10", 10, 10, "mar"), ("ising12x12", 12, 12, "mar"), ("ising12x32", 12, 32, "pr"),
             ("ising12x32", 12, 32, "mar"), ("ising16x16", 16, 16, "pr"), ("ising16x16", 16, 16, "mar"),
             ("ising20x20", 20, 20, "pr"), ("ising32x32-col", 32, 32, "pr"),
             ("ising12x12", 12, 12, "mar_tree"), ("ising12x32-col", 12, 32, "mar_tree"),
             ("ising16x16", 16, 16, "mar_tree"), ("ising20x20-col", 20, 20, "mar_tree"),
             # BASELINE config 4 restated: two-layer noisy-OR BN,
             # 50 diseases, 80 findings (3 parents each) all observed positive,
             # reference min-fill width 22
             ("noisyor50x80", 50, 80, "pr"), ("noisyor50x80", 50, 80, "mar"), ("noisyor50x80", 50, 80, "mar_tree")]
    tmp = tempfile.mkdtemp()
    for name, r, c, kind in cases:
        if args.only and args.only not in name:
            continue
        ev, evid = {}, "-"
        if name.startswith("noisyor"):
            md = synth.noisy_or_bn(r, c, 3, seed=0)
            ev = {r + i: 1 for i in range(c)}
            evid = os.path.join(tmp, name + ".uai.evid")
            synth.write_evidence(ev, evid)
        else:
            md = synth.ising_grid(r, c, seed=0)
        path = os.path.join(tmp, name + ".uai")
        synth.write_uai(md, path)
        m = bnpp.Model.load(path)
        order = None
        if name.endswith("-col"):          # width-32 column sweep (SURVEY 8(d), config 3 restated)
            order = [rr * c + cc for cc in range(c) for rr in range(r)]
        for dtype in (bnpp.F32, bnpp.F64):
            if name.startswith("ising32x32") and dtype == bnpp.F64:
                continue
            rec = {"instance": name, "task": kind.upper(), "dtype": "f32" if dtype == bnpp.F32 else "f64"}
            t0 = time.perf_counter()
            if kind == "pr":
                lz, _, up = bnpp.partition(ctx, m, ev, "mf", dtype, order=order)
                rec["log10Z"] = lz
            elif kind == "mar":
                marg, up = bnpp.marginals(ctx, m, ev, "mf", dtype)
                rec["p0"] = marg[0]
            else:
                marg, up = bnpp.marginals_tree(ctx, m, ev, "mf", dtype, order=order)
                rec["p0"] = marg[0]
            rec["gpu_uptime_ms"] = up
            rec["gpu_call_ms"] = (time.perf_counter() - t0) * 1e3
            job = bnpp.Job(ctx, m, kind, evidence=ev, heuristic="mf", dtype=dtype, order=order)
            job.launch()
            job.results()
            ts = []
            for _ in range(3):
                t1 = time.perf_counter()
                job.launch()
                job.results()
                ts.append((time.perf_counter() - t1) * 1e3)
            rec["gpu_launch_ms"] = min(ts)
            rec.update({"entries": job.entries, "levels": job.levels, "buckets": job.buckets, "width": job.width,
                        "arena_GB": job.arena_bytes / 1e9, "alg_GB": job.alg_bytes / 1e9,
                        "batches": job.batches})
            job.close()
            big_mar = kind == "mar" and r * c > 256 and not name.startswith("noisyor")
            if args.ref and dtype == bnpp.F64 and kind != "mar_tree" and not name.endswith("-col") and not big_mar:
                # the reference's MAR on the noisy-OR net is 130 VEs of width 22 (~6 min)
                tmo = max(args.ref_timeout, 900) if name.startswith("noisyor") else args.ref_timeout
                rec["ref_ms"] = ref_time(kind, path, tmo, evid)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
