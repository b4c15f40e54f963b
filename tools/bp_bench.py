#!/usr/bin/env python3
"""Loopy BP (-sp) timing: device (bnpp_sum_product, one workgroup) against the
reference's own FactorGraph (oracle/_ref/ref_harness sp, compiled from the
reference sources, one core), both on the box running this script.

    python tools/bp_bench.py > gpurun_out/bp_bench.jsonl
"""
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))
import bnpp  # noqa: E402

MODELS = os.path.join(REPO, "tests", "golden", "models")
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
CASES = [("alarm.uai", 0.001), ("insurance.uai", 0.001), ("hailfinder.uai", 0.001), ("win95pts.uai", 0.001),
         ("hepar2.uai", 0.001), ("andes.uai", 0.001), ("Water.uai", 0.001), ("pathfinder.uai", 0.001),
         ("network.uai", 0.001), ("ising10x10.uai", 1e-6), ("ising12x12.uai", 1e-6), ("grid3x3.uai", 0.001)]


def ref_ms(path, eps):
    if not os.path.exists(HARNESS):
        return None
    out = subprocess.run([HARNESS, "sp", path, "10000", repr(eps)], capture_output=True, text=True, timeout=120,
                         check=True).stdout
    kv = dict(line.split()[:2] for line in out.splitlines() if line.startswith(("uptime_ms", "iterations")))
    return float(kv["uptime_ms"]), int(kv["iterations"])


def main():
    ctx = bnpp.Context(0)
    for name, eps in CASES:
        path = os.path.join(MODELS, name)
        m = bnpp.Model.load(path)
        bnpp.sum_product(ctx, m, 10000, eps)                     # warm-up (module load)
        ts, it = [], 0
        for _ in range(5):
            _, it, up = bnpp.sum_product(ctx, m, 10000, eps)
            ts.append(up)
        rec = {"instance": name, "task": "MAR -sp", "eps": eps, "iterations": it, "gpu_uptime_ms": statistics.median(ts)}
        r = ref_ms(path, eps)
        if r:
            rec["ref_ms"], rec["ref_iterations"] = r
            rec["speedup"] = r[0] / rec["gpu_uptime_ms"]
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
