"""Synthetic UAI models and bucket shapes (SURVEY.md §8(d) generator spec).

Models are plain dicts so they can be written as UAI text, handed to the C-ABI
(`bnpp_model_from_arrays`) or to the oracle with the same numbers:

    {"type": "MARKOV"|"BAYES", "cards": [int], "scopes": [[int]], "values": [[float]]}

Values are rounded through "%.6g" so that the in-memory model and the UAI file
written from it are bit-identical.
"""
from __future__ import annotations

import math
import random


def _r6(x: float) -> float:
    return float("%.6g" % x)


def ising_grid(rows: int, cols: int, seed: int = 0) -> dict:
    """R x C binary Ising grid: var id = r*C + c; R*C unary factors (row-major),
    then horizontal pairs (i, i+1), then vertical pairs (i, i+C).
    unary = [e^h, e^-h], pairwise = [e^J, e^-J, e^-J, e^J], h, J ~ U(-1, 1)
    drawn from random.Random(seed), one draw per factor in list order."""
    rng = random.Random(seed)
    n = rows * cols
    scopes, values = [], []
    for i in range(n):
        h = rng.uniform(-1.0, 1.0)
        scopes.append([i])
        values.append([_r6(math.exp(h)), _r6(math.exp(-h))])
    pairs = [(r * cols + c, r * cols + c + 1) for r in range(rows) for c in range(cols - 1)]
    pairs += [(r * cols + c, (r + 1) * cols + c) for r in range(rows - 1) for c in range(cols)]
    for a, b in pairs:
        j = rng.uniform(-1.0, 1.0)
        e, ne = _r6(math.exp(j)), _r6(math.exp(-j))
        scopes.append([a, b])
        values.append([e, ne, ne, e])
    return {"type": "MARKOV", "cards": [2] * n, "scopes": scopes, "values": values}


def peaked_grid(rows: int, cols: int, log2_eps: int = 10, seed: int = 0) -> dict:
    """R x C binary grid whose bucket products peak far below 1 (the factor
    list as ising_grid's).  unary = [a, eps b] prefers x = 0, the vertical pair
    (v, v+C) = [eps c, eps d, e, f] penalises x_v = 0, the horizontal pair is
    U(0.5, 1): on a column sweep the bucket of every variable above the last
    row holds all three, so its product is <= eps everywhere (eps = 2^-log2_eps)
    although every table's maximum is near 1 -- a run of F fused buckets then
    carries a power-of-two rescale of about F * log2_eps."""
    rng = random.Random(seed)
    eps = 2.0 ** -log2_eps
    u = lambda: rng.uniform(0.5, 1.0)
    n = rows * cols
    scopes, values = [], []
    for i in range(n):
        scopes.append([i])
        values.append([_r6(u()), _r6(eps * u())])
    pairs = [(r * cols + c, r * cols + c + 1) for r in range(rows) for c in range(cols - 1)]
    for a, b in pairs:
        scopes.append([a, b])
        values.append([_r6(u()) for _ in range(4)])
    vpairs = [(r * cols + c, (r + 1) * cols + c) for r in range(rows - 1) for c in range(cols)]
    for a, b in vpairs:
        scopes.append([a, b])
        values.append([_r6(eps * u()), _r6(eps * u()), _r6(u()), _r6(u())])
    return {"type": "MARKOV", "cards": [2] * n, "scopes": scopes, "values": values}


def potts_grid(rows: int, cols: int, k: int = 4, seed: int = 0) -> dict:
    """R x C k-state Potts grid: unary = exp(U(-1,1)) per state; pairwise =
    e^J on the diagonal, e^-J elsewhere."""
    rng = random.Random(seed)
    n = rows * cols
    scopes, values = [], []
    for i in range(n):
        scopes.append([i])
        values.append([_r6(math.exp(rng.uniform(-1.0, 1.0))) for _ in range(k)])
    pairs = [(r * cols + c, r * cols + c + 1) for r in range(rows) for c in range(cols - 1)]
    pairs += [(r * cols + c, (r + 1) * cols + c) for r in range(rows - 1) for c in range(cols)]
    for a, b in pairs:
        j = rng.uniform(-1.0, 1.0)
        e, ne = _r6(math.exp(j)), _r6(math.exp(-j))
        scopes.append([a, b])
        values.append([e if x == y else ne for x in range(k) for y in range(k)])
    return {"type": "MARKOV", "cards": [k] * n, "scopes": scopes, "values": values}


def noisy_or_bn(n_diseases: int, n_findings: int, parents_per_finding: int, seed: int = 0) -> dict:
    """Two-layer noisy-OR BN (Promedas-style, BASELINE config 4).  Factor i is
    the CPT of variable i with the child first (model.cpp:113-114): diseases
    0..D-1 are roots with prior [1-p, p]; findings D.. have `parents_per_finding`
    disease parents and P(f=0 | pa) = (1-leak) * prod_{j on} (1-q_j)."""
    rng = random.Random(seed)
    cards = [2] * (n_diseases + n_findings)
    scopes, values = [], []
    for d in range(n_diseases):
        p = _r6(rng.uniform(0.01, 0.2))
        scopes.append([d])
        values.append([_r6(1 - p), p])
    for f in range(n_findings):
        fid = n_diseases + f
        pa = sorted(rng.sample(range(n_diseases), parents_per_finding))
        q = [rng.uniform(0.2, 0.9) for _ in pa]
        leak = rng.uniform(0.001, 0.05)
        tab0, tab1 = [], []
        for idx in range(1 << len(pa)):
            off = 1.0 - leak
            for j in range(len(pa)):
                if (idx >> (len(pa) - 1 - j)) & 1:
                    off *= 1.0 - q[j]
            off = _r6(off)
            tab0.append(off)
            tab1.append(_r6(1.0 - off))
        scopes.append([fid] + pa)
        values.append(tab0 + tab1)       # child is the slowest variable
    return {"type": "BAYES", "cards": cards, "scopes": scopes, "values": values}


def write_uai(model: dict, path: str) -> None:
    with open(path, "w") as f:
        f.write(model["type"] + "\n")
        f.write("%d\n" % len(model["cards"]))
        f.write(" ".join(str(c) for c in model["cards"]) + "\n")
        f.write("%d\n" % len(model["scopes"]))
        for s in model["scopes"]:
            f.write("%d %s\n" % (len(s), " ".join(str(v) for v in s)))
        for vals in model["values"]:
            f.write("\n%d\n%s\n" % (len(vals), " ".join("%.17g" % v for v in vals)))


def write_evidence(ev: dict, path: str) -> None:
    with open(path, "w") as f:
        f.write("1\n%d %s\n" % (len(ev), " ".join("%d %d" % (k, v) for k, v in sorted(ev.items()))))


def read_uai(path: str) -> dict:
    """UAI reader with the reference's token rules (io.cpp:14-100)."""
    toks = []
    with open(path) as f:
        for line in f:
            for t in line.split():
                if t.startswith("#"):
                    break
                toks.append(t)
    it = iter(toks)
    typ = next(it)
    n = int(next(it))
    cards = [int(next(it)) for _ in range(n)]
    nf = int(next(it))
    scopes = []
    for _ in range(nf):
        w = int(next(it))
        scopes.append([int(next(it)) for _ in range(w)])
    values = []
    for _ in range(nf):
        sz = int(next(it))
        values.append([float(next(it)) for _ in range(sz)])
    return {"type": typ, "cards": cards, "scopes": scopes, "values": values}


def read_evidence(path: str) -> dict:
    """read_uai_evidence (io.cpp:157-180): read only when the first integer is 1."""
    toks = []
    with open(path) as f:
        for line in f:
            for t in line.split():
                if t.startswith("#"):
                    break
                toks.append(t)
    ev = {}
    if toks and int(toks[0]) == 1:
        m = int(toks[1])
        for i in range(m):
            ev[int(toks[2 + 2 * i])] = int(toks[3 + 2 * i])
    return ev
