#!/usr/bin/env python3
"""Where a modelled sliced run idles (rocprofv3 kernel trace, tools/gpu_r6v.sh):
the trace is cut into calls at > 50 ms (argv[2]) with no kernel, and for each call this
prints its span, the time with no working kernel (delay_kernel, which holds a
stream for an exchange's modelled xGMI time, does not count as work), and how
much of that idle time has 0 / 1 / 2 lanes inside a delay.

    python tools/idle_gaps.py gpurun_out/r6v_alt/sliced/.../sliced_kernel_trace.csv"""
import csv
import sys


GAP = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 50e6      # ms of no kernel between calls


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "delay_kernel" in r["Kernel_Name"]) for r in rows)
    calls, cur, mx = [], [ev[0]], ev[0][1]
    for e in ev[1:]:
        if e[0] - mx > GAP:
            calls.append(cur)
            cur = []
        cur.append(e)
        mx = max(mx, e[1])
    calls.append(cur)
    for i, c in enumerate(calls):
        pts = sorted([(s, 1, d) for s, _, d in c] + [(e, -1, d) for _, e, d in c])
        work = delay = 0
        last = pts[0][0]
        idle = {0: 0, 1: 0, 2: 0}
        for t, dd, isd in pts:
            if work == 0:
                idle[min(delay, 2)] += t - last
            last = t
            if isd:
                delay += dd
            else:
                work += dd
        span = max(e for _, e, _ in c) - c[0][0]
        n_delay = sum(1 for _, _, d in c if d)
        print("call %d: %d kernels (%d delays), span %.1f ms, no working kernel %.1f ms "
              "(0 / 1 / 2 lanes in a delay: %.1f / %.1f / %.1f ms)" % (
                  i, len(c), n_delay, span / 1e6, sum(idle.values()) / 1e6, idle[0] / 1e6, idle[1] / 1e6,
                  idle[2] / 1e6))


if __name__ == "__main__":
    main()
