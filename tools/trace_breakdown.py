#!/usr/bin/env python3
"""Kernel-time breakdown of a rocprofv3 kernel trace (*_kernel_trace.csv):
the last of the runs separated by > 50 ms of idle GPU (--last), its span,
busy union, kernel time per kernel name, how long 0 / 1 / 2 kernels ran at
once (two-lane schedules), and the idle gaps inside it."""
import collections
import csv
import re
import sys


def name(n):
    n = n.replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n).replace("void bnpp::", "")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name(r["Kernel_Name"])) for r in rows)
    starts, mx = [0], ev[0][1]
    for i in range(1, len(ev)):
        if ev[i][0] - mx > 50e6:
            starts.append(i)
        mx = max(mx, ev[i][1])
    seg = ev[starts[-1]:]
    print("runs (split at > 50 ms idle): %d; the last: %d kernels" % (len(starts), len(seg)))
    t0, t1 = seg[0][0], max(e[1] for e in seg)
    pts = sorted([(s, 1) for s, _, _ in seg] + [(e, -1) for _, e, _ in seg])
    lvl, last, hist = 0, pts[0][0], collections.Counter()
    for t, d in pts:
        hist[lvl] += t - last
        last, lvl = t, lvl + d
    print("span %.1f ms; time with 0/1/2/3 kernels running: %s ms" % (
        (t1 - t0) / 1e6, {k: round(v / 1e6, 1) for k, v in sorted(hist.items())}))
    agg = collections.defaultdict(lambda: [0, 0.0])
    for s, e, n in seg:
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e6
    for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
        print("%-60s %5d %9.2f ms" % (n[:60], c, t))


if __name__ == "__main__":
    main()
