#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace into calls (gaps > --gap ms between kernels)
and summarise each: span, kernel busy time, idle gaps, per-kernel averages.
Used to compare a cold call with a warm one (tools/cold_probe.sh).

    python tools/trace_calls.py KERNEL_TRACE.csv > calls.json
"""
import argparse
import collections
import csv
import json
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap", type=float, default=50.0, help="ms of idle GPU that separates two calls")
    args = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(args.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), re.sub(r"\(.*", "", r["Kernel_Name"])))
    rows.sort()
    calls, cur = [], []
    for r in rows:
        if cur and (r[0] - cur[-1][1]) / 1e6 > args.gap:
            calls.append(cur)
            cur = []
        cur.append(r)
    if cur:
        calls.append(cur)
    out = []
    for i, c in enumerate(calls):
        busy = sum(e - s for s, e, _ in c) / 1e6
        span = (c[-1][1] - c[0][0]) / 1e6
        per = collections.defaultdict(list)
        for s, e, k in c:
            per[k].append((e - s) / 1e6)
        top = sorted(per.items(), key=lambda kv: -sum(kv[1]))[:8]
        gaps = sorted(((c[j + 1][0] - c[j][1]) / 1e6, j) for j in range(len(c) - 1))[-5:]
        out.append({"call": i, "kernels": len(c), "span_ms": span, "busy_ms": busy, "idle_ms": span - busy,
                    "first_start_ns": c[0][0],
                    "gap_before_ms": (c[0][0] - calls[i - 1][-1][1]) / 1e6 if i else None,
                    "largest_gaps_ms": [round(g, 3) for g, _ in gaps],
                    "first10_ms": [round((e - s) / 1e6, 3) for s, e, _ in c[:10]],
                    "top": [{"kernel": k[:90], "n": len(v), "total_ms": sum(v), "avg_ms": sum(v) / len(v),
                             "max_ms": max(v)} for k, v in top]})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
