#!/usr/bin/env python3
"""Bucket shapes of a VE run (host only): for each bucket of the min-fill
elimination (BN::variable_elimination's bucket assignment, model.cpp:394-438)
its factor-entries (prod card over the union scope, summed variable
included), the summed variable's card, and the inputs' sizes.  Used to ask
whether any bucket of the reference's large-card networks is a GEMM-shaped
contraction MFMA could serve: a product of two large inputs
sharing the summed variable.

    python tools/bucket_shapes.py Mildew.uai Barley.uai pathfinder.uai
"""
import json
import os
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))
import bnpp  # noqa: E402

MODELS = os.path.join(REPO, "tests", "golden", "models")


def prod(cards, scope):
    p = 1
    for v in scope:
        p *= cards[v]
    return p


def uai_scopes(path):
    """scopes of a UAI file (io.cpp:43-100 token rules: '#' comments)"""
    toks = []
    with open(path) as f:
        for line in f:
            for t in line.split():
                if t.startswith("#"):
                    break
                toks.append(t)
    i = 1
    nv = int(toks[i]); i += 1
    i += nv
    nf = int(toks[i]); i += 1
    scopes = []
    for _ in range(nf):
        w = int(toks[i]); i += 1
        scopes.append([int(x) for x in toks[i:i + w]]); i += w
    return scopes


def shapes(name, ev_name=None):
    m = bnpp.Model.load(os.path.join(MODELS, name))
    ev = bnpp.load_evidence(os.path.join(MODELS, ev_name)) if ev_name else {}
    cards = m.cards
    m.scopes = uai_scopes(os.path.join(MODELS, name))
    order, width = bnpp.ordering(m, ev, "mf")
    rank = {v: i for i, v in enumerate(order)}
    facs = [[v for v in s if v not in ev] for s in m.scopes]
    buckets = {v: [] for v in order}
    for s in facs:
        vs = [v for v in s if v in rank]
        if vs:
            buckets[min(vs, key=lambda v: rank[v])].append(s)
    rows = []
    for v in order:
        ins = buckets[v]
        union = []
        for s in ins:
            union += [x for x in s if x not in union]
        ent = prod(cards, union)
        out = [x for x in union if x != v]
        sizes = sorted((prod(cards, s) for s in ins), reverse=True)
        rows.append({"var": v, "card": cards[v], "entries": ent, "n_in": len(ins),
                     "big_inputs": sizes[:2], "out": prod(cards, out)})
        if out:
            nxt = min(out, key=lambda x: rank[x])
            buckets[nxt].append(out)
    rows.sort(key=lambda r: -r["entries"])
    tot = sum(r["entries"] for r in rows)
    # GEMM-shaped: two inputs each >= 4096 entries sharing the summed variable
    gemm = [r for r in rows if len(r["big_inputs"]) > 1 and r["big_inputs"][1] >= 4096]
    return {"model": name, "width": width, "buckets": len(rows), "factor_entries": tot,
            "top5": rows[:5], "top5_share": sum(r["entries"] for r in rows[:5]) / tot,
            "gemm_shaped": len(gemm), "gemm_entries_share": sum(r["entries"] for r in gemm) / tot,
            "max_card": max(cards)}


if __name__ == "__main__":
    for a in sys.argv[1:]:
        n, _, e = a.partition(":")
        print(json.dumps(shapes(n, e or None)), flush=True)
