#!/usr/bin/env python3
"""BASELINE config 4 (Promedas-style noisy-OR BN, 50 diseases -> 80 findings,
all findings observed, reference min-fill width 22) from one run: GPU PR,
per-target MAR (BN::marginals as the reference runs it, model.cpp:326-334)
and bucket-tree MAR, fp64 and fp32, median of --reps warm calls (wall-clock of
the ABI call: ordering + planning + device run + fetch), beside the
reference's measured PR and per-target MAR from tests/golden/config4_golden.json.

    python tools/config4_bench.py > gpurun_out/config4_bench.jsonl
"""
import json
import os
import statistics
import sys
import time

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))
import bnpp  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")


def timed(fn, reps):
    fn()                                                   # cold call (kernels loaded, arena cached)
    ts = []
    out = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return statistics.median(ts), out


def main():
    reps = 5
    with open(os.path.join(GOLDEN, "config4_golden.json")) as f:
        g = json.load(f)
    m = bnpp.Model.load(os.path.join(GOLDEN, "models", g["model"]))
    ev = bnpp.load_evidence(os.path.join(GOLDEN, "models", g["evidence"]))
    ctx = bnpp.Context(0)
    rec = {"model": g["model"], "width": g["ref_width"], "ref_pr_ms": g["pr"]["ref_uptime_ms"],
           "ref_mar_ms_sum": g["ref_mar_ms_sum"], "ref_note": g["note"]}
    for dt, name in ((bnpp.F64, "f64"), (bnpp.F32, "f32")):
        ms, (lz, _, _) = timed(lambda: bnpp.partition(ctx, m, ev, "mf", dt), reps)
        rec["pr_ms_" + name] = ms
        rec["pr_log10Z_err_" + name] = abs(lz - g["pr"]["log10Z"])
        ms, (marg, _) = timed(lambda: bnpp.marginals(ctx, m, ev, "mf", dt), reps)
        rec["mar_per_target_ms_" + name] = ms
        err = max(abs(a - b) for t, r in g["marginals"].items() for a, b in zip(marg[int(t)], r["values"]))
        rec["mar_per_target_max_err_" + name] = err
        ms, (marg, _) = timed(lambda: bnpp.marginals_tree(ctx, m, ev, "mf", dt), reps)
        rec["mar_tree_ms_" + name] = ms
        err = max(abs(a - b) for t, r in g["marginals"].items() for a, b in zip(marg[int(t)], r["values"]))
        rec["mar_tree_max_err_" + name] = err
    rec["speedup_pr_f64"] = rec["ref_pr_ms"] / rec["pr_ms_f64"]
    rec["speedup_mar_per_target_f64"] = rec["ref_mar_ms_sum"] / rec["mar_per_target_ms_f64"]
    rec["speedup_mar_tree_f64"] = rec["ref_mar_ms_sum"] / rec["mar_tree_ms_f64"]
    print(json.dumps(rec), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
