#!/usr/bin/env python3
"""HBM bytes per dispatch, per kernel, from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, separate runs of the same program), with the
gfx950 correction of MI355X_MICROARCH.md (HBM): FETCH_SIZE counts half the
bytes of wide coalesced streaming reads -> read bytes = 2 * FETCH_SIZE KiB;
WRITE_SIZE is exact for 16-B-per-lane streaming stores.

The chain runs of a column sweep read one message and write one of the same
size (a sweep bucket swaps one variable for another), so the algorithmic read
bytes equal the write bytes; `read_over_write` is then the over-fetch ratio.

    python tools/pmc_kernels.py FETCH.csv WRITE.csv > pmc.json
"""
import collections
import csv
import json
import re
import sys


def load(path, counter):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        per[re.sub(r"\(.*", "", r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = []
    for k in sorted(set(fetch) | set(write), key=lambda k: -sum(fetch.get(k, [0])) - sum(write.get(k, [0]))):
        f, w = fetch.get(k, []), write.get(k, [])
        rd = 2 * 1024 * sum(f) / max(len(f), 1)
        wr = 1024 * sum(w) / max(len(w), 1)
        # the big dispatches only (messages of >= 1 GiB written): the steady state of the sweep
        big = [(2 * 1024 * a, 1024 * b) for a, b in zip(f, w) if 1024 * b >= 2 ** 30] if len(f) == len(w) else []
        rec = {"kernel": k[:120], "dispatches": [len(f), len(w)], "read_bytes_avg": rd, "write_bytes_avg": wr,
               "total_GB": (2 * 1024 * sum(f) + 1024 * sum(w)) / 1e9,
               "read_over_write": rd / wr if wr else None}
        if big:
            rec["big_dispatches"] = len(big)
            rec["big_read_avg"] = sum(a for a, _ in big) / len(big)
            rec["big_write_avg"] = sum(b for _, b in big) / len(big)
            rec["big_read_over_write"] = rec["big_read_avg"] / rec["big_write_avg"]
        out.append(rec)
    print(json.dumps({"correction": "read = 2*FETCH_SIZE*1024 (gfx950 wide-read undercount), write = WRITE_SIZE*1024; "
                                    "separate --pmc passes", "kernels": out}, indent=1))


if __name__ == "__main__":
    main()
