#!/usr/bin/env python3
"""Bytes a plan moves, by kernel kind, from a BNPP_DUMP_PLAN dump (stderr of
any planning call, e.g. bnpp.plan_tree_sliced): chain runs 2 x eb x entries
(+ lam for a fused belief), exchange pack / unpack read + write, other buckets
estimated from their dims rows.  Usage: tools/plan_bytes.py dump.txt [eb]"""
import collections
import re
import sys


def main():
    path = sys.argv[1]
    eb = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    tot, cnt = collections.Counter(), collections.Counter()
    for line in open(path):
        m = re.search(r"chain F=(\d+) form=(\d+).* tiles=(\d+)", line)
        if m:
            F, form, t = int(m[1]), int(m[2]), int(m[3])
            bel = "belief" in line
            key = "chain F=%d form=%d%s" % (F, form, " bel" if bel else "")
            tot[key] += (3 if bel else 2) * t * 2 ** F * eb
            cnt[key] += 1
            continue
        m = re.search(r"xchg kind=(\d+) mode=(\d+).* entries=(\d+)", line)
        if m:
            k, e = int(m[1]), int(m[3])
            key = "xchg %s" % {1: "sync", 2: "pack", 3: "comm", 4: "unpack"}.get(k, k)
            tot[key] += 2 * e * eb if k in (2, 4) else 0
            cnt[key] += 1
            continue
        if "dims:" not in line:
            continue
        m = re.search(r"n_in=(\d+) k=(\d+)", line)
        nin, k = int(m[1]), int(m[2])
        es = [int(x) for x in re.search(r"es:([-\d,]+)", line)[1].split(",")]
        out, insz = 1, [1] * nin
        for card, st in re.findall(r"\[(\d+):([-\d,]+)\]", line):
            st = [int(x) for x in st.split(",")]
            out *= int(card)
            for q in range(nin):
                if st[q]:
                    insz[q] *= int(card)
        b = eb * (out + sum(s * (k if es[q] else 1) for q, s in enumerate(insz)))
        key = "bucket n_in=%d k=%d" % (nin, k) if b > 1e9 else "buckets < 1 GB"
        tot[key] += b
        cnt[key] += 1
    for key in sorted(tot, key=lambda x: -tot[x]):
        print("%-28s n=%5d %9.1f GB" % (key, cnt[key], tot[key] / 1e9))
    print("total %.1f GB" % (sum(tot.values()) / 1e9))


if __name__ == "__main__":
    main()
