#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Run in the build container (needs /root/reference and `make -C oracle ref`):

    python tests/golden/make_golden.py          # everything
    python tests/golden/make_golden.py sp       # loopy BP fixtures only (sp_golden.json)
    python tests/golden/make_golden.py corpus   # larger networks' PR (corpus_golden.json)
    python tests/golden/make_golden.py config4  # noisy-OR 50x80, width 22 (config4_golden.json)
    python tests/golden/make_golden.py cli      # reference bn / mn stdout (cli_golden.json)
    python tests/golden/make_golden.py query    # BN::query_ve answers (query_golden.json)

It
  1. copies the reference's own model + fixture files that the tests use into
     tests/golden/models/ (data: .uai models, .evid evidence, .PR/.MAR outputs),
  2. writes the synthetic models (bn-pp_amd/python/bnpp/synth.py) next to them,
  3. runs oracle/_ref/ref_harness (the reference compiled from its sources) for
     PR / MAR / orderings / single-op known-answer tests, and
  4. stores inputs and outputs as JSON (values printed with %.17g).
Nothing here is needed at test time except the JSON and model files it writes.
"""
from __future__ import annotations

import json
import os
import random
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.normpath(os.path.join(HERE, "..", ".."))
REF_MODELS = "/root/reference/models"
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
MODELS = os.path.join(HERE, "models")
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))
from bnpp import synth  # noqa: E402

COPY = {
    "markovnets": ["grid3x3.uai", "grid3x3-PR.uai.evid", "grid3x3-MAR.uai.evid", "grid3x3.uai.PR", "grid3x3.uai.MAR",
                   "network.uai", "network.uai.evid", "network.uai.PR", "network.uai.MAR"],
    "bayesnets": ["asia.uai", "asia.uai.evid", "cancer.uai", "earthquake.uai", "child.uai", "alarm.uai",
                  "insurance.uai", "win95pts.uai", "hailfinder.uai", "hepar2.uai", "andes.uai", "Water.uai",
                  "pathfinder.uai"],
}
# the reference's larger networks (corpus bench, tools/corpus_bench.py)
CORPUS = ["Pigs.uai", "Link.uai", "Munin1.uai", "Munin2.uai", "Munin3.uai", "Munin4.uai", "Barley.uai",
          "Mildew.uai", "Diabetes.uai"]


def run(*args, timeout=900):
    out = subprocess.run([HARNESS] + [str(a) for a in args], check=True, capture_output=True, text=True,
                         timeout=timeout)
    return out.stdout


def parse_kv(text):
    d = {}
    for line in text.splitlines():
        parts = line.split()
        if len(parts) == 2:
            d[parts[0]] = float(parts[1])
    return d


def parse_factors(text):
    """lines 'TAG w ids.. | size partition | values..' -> {TAG: {...}}"""
    res = {}
    for line in text.splitlines():
        if "|" not in line:
            continue
        head, mid, vals = line.split("|")
        h = head.split()
        tag, w = h[0], int(h[1])
        size, part = mid.split()
        res[tag] = {"scope": [int(x) for x in h[2:2 + w]], "size": int(size), "partition": float(part),
                    "values": [float(x) for x in vals.split()]}
    return res


def model_path(name):
    return os.path.join(MODELS, name)


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the reference first: make -C oracle ref")
    os.makedirs(MODELS, exist_ok=True)
    for sub, names in COPY.items():
        for n in names:
            shutil.copyfile(os.path.join(REF_MODELS, sub, n), model_path(n))

    # synthetic instances (SURVEY.md §8(d) generator)
    synthetic = {}
    for n in (4, 5, 6, 8, 10, 12):
        synthetic["ising%dx%d.uai" % (n, n)] = synth.ising_grid(n, n, seed=0)
    synthetic["ising12x32.uai"] = synth.ising_grid(12, 32, seed=0)
    synthetic["potts6x6.uai"] = synth.potts_grid(6, 6, k=4, seed=0)
    synthetic["potts4x5k3.uai"] = synth.potts_grid(4, 5, k=3, seed=1)
    synthetic["noisyor_30_40.uai"] = synth.noisy_or_bn(30, 40, 3, seed=0)
    for name, m in synthetic.items():
        synth.write_uai(m, model_path(name))
    # deterministic evidence for the BNs: every 5th variable set to 0 (and 1 for odd ids)
    rng = random.Random(7)
    bn_ev = {}
    for n in ("cancer.uai", "earthquake.uai", "child.uai", "alarm.uai", "insurance.uai", "hailfinder.uai",
              "noisyor_30_40.uai"):
        m = synth.read_uai(model_path(n))
        ev = {}
        for v in range(len(m["cards"])):
            if rng.random() < 0.2:
                ev[v] = rng.randrange(m["cards"][v])
        name = n + ".evid"
        synth.write_evidence(ev, model_path(name))
        bn_ev[n] = name
    ising_ev = {}
    for n in (6, 8):
        ev = {0: 1, n * n // 2: 0, n * n - 1: 1}
        name = "ising%dx%d.uai.evid" % (n, n)
        synth.write_evidence(ev, model_path(name))
        ising_ev["ising%dx%d.uai" % (n, n)] = name

    ve = {"pr": [], "mar": [], "width": []}
    pr_cases = [("grid3x3.uai", "grid3x3-PR.uai.evid", "mf"), ("grid3x3.uai", "grid3x3-PR.uai.evid", "given"),
                ("grid3x3.uai", "-", "mf"), ("network.uai", "-", "mf"), ("asia.uai", "asia.uai.evid", "given"),
                ("asia.uai", "asia.uai.evid", "mf"), ("potts6x6.uai", "-", "mf"), ("potts4x5k3.uai", "-", "wmf"),
                ("ising12x32.uai", "-", "mf")]
    for n in (4, 5, 6, 8, 10, 12):
        pr_cases.append(("ising%dx%d.uai" % (n, n), "-", "mf"))
    pr_cases += [("ising6x6.uai", "ising6x6.uai.evid", "md"), ("ising8x8.uai", "ising8x8.uai.evid", "wmf")]
    for n, e in bn_ev.items():
        pr_cases.append((n, e, "mf"))
    for n in ("pathfinder.uai", "Water.uai", "hepar2.uai", "win95pts.uai", "andes.uai"):
        pr_cases.append((n, "-", "mf"))
    for model, ev, h in pr_cases:
        r = parse_kv(run("pr", model_path(model), model_path(ev) if ev != "-" else "-", h))
        ve["pr"].append({"model": model, "evidence": ev, "heuristic": h, "Z": r["Z"], "log10Z": r["log10Z"],
                         "ref_uptime_ms": r["uptime_ms"]})
        print("pr", model, ev, h, r["log10Z"])

    mar_cases = [("grid3x3.uai", "grid3x3-MAR.uai.evid", "mf"), ("network.uai", "-", "mf"),
                 ("asia.uai", "-", "mf"), ("asia.uai", "asia.uai.evid", "given"), ("ising4x4.uai", "-", "mf"),
                 ("ising6x6.uai", "ising6x6.uai.evid", "mf"), ("ising8x8.uai", "-", "md"),
                 ("potts4x5k3.uai", "-", "mf"), ("child.uai", bn_ev["child.uai"], "mf"),
                 ("alarm.uai", bn_ev["alarm.uai"], "wmf"), ("noisyor_30_40.uai", bn_ev["noisyor_30_40.uai"], "mf")]
    for model, ev, h in mar_cases:
        txt = run("mar", model_path(model), model_path(ev) if ev != "-" else "-", h)
        fs = parse_factors(txt)
        marg = {}
        for tag, f in fs.items():
            marg[int(tag[1:])] = {"scope": f["scope"], "values": f["values"]}
        up = parse_kv(txt).get("uptime_ms")
        ve["mar"].append({"model": model, "evidence": ev, "heuristic": h, "marginals": marg, "ref_uptime_ms": up})
        print("mar", model, ev, h, len(marg))

    for model in ("ising8x8.uai", "ising10x10.uai", "ising12x12.uai", "ising12x32.uai", "network.uai", "alarm.uai",
                  "potts6x6.uai"):
        for h in ("mf", "wmf", "md"):
            txt = run("width", model_path(model), h)
            w = int(txt.split()[1])
            ve["width"].append({"model": model, "heuristic": h, "width": w})
    with open(os.path.join(HERE, "ve_golden.json"), "w") as f:
        json.dump(ve, f, indent=1)

    # ------------------------------------------------- single-op KATs
    rng = random.Random(12345)
    lines, cases = [], []
    cards = {}
    for v in range(10):
        cards[v] = rng.randint(2, 5)
        lines.append("var %d %d" % (v, cards[v]))

    def rand_scope(wmax):
        w = rng.randint(0, wmax)
        return rng.sample(range(10), w)

    def size_of(scope):
        s = 1
        for v in scope:
            s *= cards[v]
        return s

    def rand_values(scope, lo=0.05, hi=3.0):
        return [rng.uniform(lo, hi) for _ in range(size_of(scope))]

    fid = 0

    def factor(scope, values=None):
        nonlocal fid
        name = "F%d" % fid
        fid += 1
        vals = values if values is not None else rand_values(scope)
        lines.append("factor %s %d %s %s" % (name, len(scope), " ".join(map(str, scope)),
                                            " ".join("%.17g" % x for x in vals)))
        return name, scope, vals

    for t in range(60):
        a = factor(rand_scope(4))
        b = factor(rand_scope(4))
        out = "P%d" % t
        lines.append("product %s %s %s" % (out, a[0], b[0]))
        lines.append("print %s" % out)
        case = {"op": "product", "a": a[0], "b": b[0], "out": out}
        # sum out a random variable of the union (or one that is absent)
        un = a[1] + [v for v in b[1] if v not in a[1]]
        x = rng.choice(un) if un and rng.random() < 0.85 else rng.randrange(10)
        so = "S%d" % t
        lines.append("sum_out %s %s %d" % (so, out, x))
        lines.append("print %s" % so)
        cases.append(case)
        cases.append({"op": "sum_out", "a": out, "var": x, "out": so})
        # conditioning on up to 2 variables (some outside the scope)
        ev = {}
        for v in rng.sample(range(10), rng.randint(0, 3)):
            ev[v] = rng.randrange(cards[v])
        co = "C%d" % t
        lines.append("cond %s %s %d %s" % (co, a[0], len(ev), " ".join("%d %d" % kv for kv in sorted(ev.items()))))
        lines.append("print %s" % co)
        cases.append({"op": "cond", "a": a[0], "evidence": {str(k): v for k, v in ev.items()}, "out": co})
        no = "N%d" % t
        lines.append("normalize %s %s" % (no, b[0]))
        lines.append("print %s" % no)
        cases.append({"op": "normalize", "a": b[0], "out": no})
        do = "D%d" % t
        lines.append("divide %s %s %s" % (do, a[0], b[0]))
        lines.append("print %s" % do)
        cases.append({"op": "divide", "a": a[0], "b": b[0], "out": do})
    # buckets: chains of 2..5 factors then sum_out (model.cpp:414-418)
    for t in range(40):
        m = rng.randint(2, 5)
        fs = [factor(rand_scope(3)) for _ in range(m)]
        un = []
        for f in fs:
            un += [v for v in f[1] if v not in un]
        if not un:
            continue
        x = rng.choice(un)
        cur = fs[0][0]
        for i, f in enumerate(fs[1:]):
            nxt = "B%d_%d" % (t, i)
            lines.append("product %s %s %s" % (nxt, cur, f[0]))
            cur = nxt
        out = "M%d" % t
        lines.append("sum_out %s %s %d" % (out, cur, x))
        lines.append("print %s" % out)
        cases.append({"op": "bucket", "inputs": [f[0] for f in fs], "var": x, "out": out})
    factors = {}
    for line in lines:
        p = line.split()
        if p[0] == "factor":
            w = int(p[2])
            factors[p[1]] = {"scope": [int(x) for x in p[3:3 + w]], "values": [float(x) for x in p[3 + w:]]}
    opfile = os.path.join("/tmp", "bnpp_kat_ops.txt")
    with open(opfile, "w") as f:
        f.write("\n".join(lines) + "\n")
    outs = parse_factors(run("kat", opfile))
    with open(os.path.join(HERE, "kat_golden.json"), "w") as f:
        json.dump({"cards": {str(k): v for k, v in cards.items()}, "factors": factors, "cases": cases,
                   "outputs": outs}, f)
    print("kat cases", len(cases), "outputs", len(outs))


# loopy BP (-sp): BN::sum_product + marginals (model.cpp:313-317, 736-753);
# evidence is ignored by the reference on this path.  (model, max_iter, eps)
SP_CASES = [("asia.uai", 10000, 0.001), ("cancer.uai", 10000, 0.001), ("earthquake.uai", 10000, 0.001),
            ("alarm.uai", 10000, 0.001), ("alarm.uai", 10000, 1e-9), ("child.uai", 10000, 0.001),
            ("insurance.uai", 10000, 0.001), ("hailfinder.uai", 10000, 0.001), ("win95pts.uai", 10000, 0.001),
            ("hepar2.uai", 10000, 0.001), ("andes.uai", 10000, 0.001), ("Water.uai", 10000, 0.001),
            ("pathfinder.uai", 10000, 0.001), ("network.uai", 10000, 0.001), ("ising4x4.uai", 10000, 0.001),
            ("ising8x8.uai", 10000, 0.001), ("ising10x10.uai", 10000, 1e-6), ("potts4x5k3.uai", 10000, 0.001),
            ("noisyor_30_40.uai", 10000, 0.001), ("grid3x3.uai", 50, 0.001), ("asia.uai", 0, 0.001)]


def sp_golden():
    cases = []
    for model, mx, eps in SP_CASES:
        txt = run("sp", model_path(model), mx, repr(eps))
        kv = parse_kv(txt)
        marg = {int(t[1:]): f["values"] for t, f in parse_factors(txt).items()}
        cases.append({"model": model, "max_iter": mx, "eps": eps, "iterations": int(kv["iterations"]),
                      "marginals": marg, "ref_uptime_ms": kv.get("uptime_ms")})
        print("sp", model, mx, eps, int(kv["iterations"]))
    with open(os.path.join(HERE, "sp_golden.json"), "w") as f:
        json.dump({"cases": cases}, f)


def ancestral_sample(m, rng):
    """One joint sample of a BN (factor i = CPT of variable i, scope[0] = the
    child, model.cpp:104-125): evidence drawn from it has P(e) > 0."""
    cards, val = m["cards"], [-1] * len(m["cards"])
    pending = set(range(len(cards)))
    while pending:
        done = []
        for i in sorted(pending):
            sc = m["scopes"][i]
            if any(val[p] < 0 for p in sc[1:]):
                continue
            off, st = 0, 1
            for p in reversed(sc[1:]):                    # row-major, last variable fastest
                off += val[p] * st
                st *= cards[p]
            row = [m["values"][i][x * st + off] for x in range(cards[i])]
            r, acc, pick = rng.random() * sum(row), 0.0, 0
            for x, w in enumerate(row):
                acc += w
                if w > 0:
                    pick = x
                if w > 0 and r < acc:
                    break
            val[i] = pick
            done.append(i)
        assert done, "cyclic CPT structure"
        pending.difference_update(done)
    return val


def corpus_golden():
    """BN::partition (min-fill) on the reference's larger networks, without and
    (three of them) with evidence sampled from the network; the reference's own
    time is kept for the bench."""
    rng = random.Random(99)
    cases = []
    for n in CORPUS:
        shutil.copyfile(os.path.join(REF_MODELS, "bayesnets", n), model_path(n))
        evs = ["-"]
        if n in ("Pigs.uai", "Munin2.uai", "Diabetes.uai"):
            m = synth.read_uai(model_path(n))
            x = ancestral_sample(m, rng)
            ev = {v: x[v] for v in range(len(m["cards"])) if rng.random() < 0.1}
            synth.write_evidence(ev, model_path(n + ".evid"))
            evs.append(n + ".evid")
        for e in evs:
            r = parse_kv(run("pr", model_path(n), model_path(e) if e != "-" else "-", "mf", timeout=1800))
            w = int(run("width", model_path(n), "mf").split()[1])
            cases.append({"model": n, "evidence": e, "heuristic": "mf", "Z": r["Z"], "log10Z": r["log10Z"],
                          "ref_uptime_ms": r["uptime_ms"], "ref_width": w})
            print("corpus", n, e, r["log10Z"], r["uptime_ms"], w)
    with open(os.path.join(HERE, "corpus_golden.json"), "w") as f:
        json.dump({"cases": cases}, f, indent=1)


# BASELINE config 4 at its stated size: a two-layer noisy-OR
# BN, 50 diseases -> 80 findings (3 parents each), every finding observed;
# reference min-fill width 22.  Reference PR (BN::partition, model.cpp:250-301),
# three single-target conditionings Z(x_t = s), and the reference MAR of every
# disease (one VE per target, model.cpp:326-334), run as 8 parallel processes.
C4_MODEL = "noisyor_50_80.uai"
C4_TARGETS = (0, 24, 49)


def config4_golden():
    from concurrent.futures import ThreadPoolExecutor
    md = synth.noisy_or_bn(50, 80, 3, seed=0)
    synth.write_uai(md, model_path(C4_MODEL))
    rng = random.Random(50)
    ev = {v: rng.randrange(2) for v in range(50, 130)}
    synth.write_evidence(ev, model_path(C4_MODEL + ".evid"))
    path, evp = model_path(C4_MODEL), model_path(C4_MODEL + ".evid")
    cond_files = []
    for t in C4_TARGETS:
        e = dict(ev)
        e[t] = 1
        name = "/tmp/%s.t%d.evid" % (C4_MODEL, t)
        synth.write_evidence(e, name)
        cond_files.append((t, name))

    def job(spec):
        kind, arg = spec
        if kind == "pr":
            return spec, parse_kv(run("pr", path, arg, "mf", timeout=3600))
        return spec, run("mar", path, evp, "mf", *arg, timeout=3600)

    specs = [("pr", evp)] + [("pr", f) for _, f in cond_files]
    diseases = list(range(50))
    specs += [("mar", tuple(diseases[i::8])) for i in range(8)]
    with ThreadPoolExecutor(8) as ex:
        res = dict(ex.map(job, specs))
    width = int(run("width", path, "mf").split()[1])
    pr = res[("pr", evp)]
    conds = [{"target": t, "value": 1, "log10Z": res[("pr", f)]["log10Z"], "Z": res[("pr", f)]["Z"],
              "ref_uptime_ms": res[("pr", f)]["uptime_ms"]} for t, f in cond_files]
    marg, mar_ms = {}, 0.0
    for i in range(8):
        txt = res[("mar", tuple(diseases[i::8]))]
        for tag, f in parse_factors(txt).items():
            marg[int(tag[1:])] = {"scope": f["scope"], "values": f["values"]}
        mar_ms += parse_kv(txt)["uptime_ms"]
    out = {"model": C4_MODEL, "evidence": C4_MODEL + ".evid", "heuristic": "mf", "ref_width": width,
           "pr": {"Z": pr["Z"], "log10Z": pr["log10Z"], "ref_uptime_ms": pr["uptime_ms"]},
           "conditioned": conds, "marginals": marg,
           "ref_mar_ms_sum": mar_ms,
           "note": "reference MAR timed per target in 8 parallel processes (sum of their uptimes); "
                   "findings (ids 50..129) are evidence, their marginals are one-hot"}
    with open(os.path.join(HERE, "config4_golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("config4", pr["log10Z"], width, len(marg), mar_ms)


# CLI output parity (bn.cpp:224-258, mn.cpp:135-155, factor.cpp:291-321): the
# exact stdout of the reference's own `bn` and `mn` binaries (oracle/_ref,
# compiled from /root/reference/code) on the bundled models.  `bn` cases are
# argv lists (run from tests/golden/models); `mn` cases are (argv, stdin).
# Cases the reference crashes on (-mar with evidence and -mf/-wmf/-md,
# SURVEY 0.6) are left out.
CLI_BN = {
    "bn_asia_pr": ["asia.uai", "-pr"],
    "bn_asia_mar": ["asia.uai", "-mar"],
    "bn_asia_pr_mar_mf": ["asia.uai", "-pr", "-mar", "-mf"],
    "bn_asia_ev_pr_mar": ["asia.uai", "asia.uai.evid", "-pr", "-mar"],
    "bn_asia_mar_sp": ["asia.uai", "-mar", "-sp"],
    "bn_alarm_ev_pr_mf": ["alarm.uai", "alarm.uai.evid", "-pr", "-mf"],
    "bn_alarm_ev_pr_mar": ["alarm.uai", "alarm.uai.evid", "-pr", "-mar"],
    "bn_child_pr_mar_wmf": ["child.uai", "-pr", "-mar", "-wmf"],
    "bn_hailfinder_ev_pr_md": ["hailfinder.uai", "hailfinder.uai.evid", "-pr", "-md"],
    "bn_insurance_ve_mar_mf": ["insurance.uai", "-mar", "-ve", "-mf"],
}
CLI_MN = {
    "mn_grid3x3_pr_mar": (["grid3x3.uai", "grid3x3-PR.uai.evid"], "PR\nMAR\nquit\n"),
    "mn_grid3x3_mar_pr": (["grid3x3.uai", "grid3x3-MAR.uai.evid"], "MAR\npartition\nfoo\nquit\n"),
    "mn_grid3x3_verbose": (["grid3x3.uai", "grid3x3-PR.uai.evid", "-v"], "PR\nquit\n"),
    "mn_network_verbose": (["network.uai", "network.uai.evid", "-v"], "quit\n"),
}


def cli_golden():
    out_dir = os.path.join(HERE, "cli")
    os.makedirs(out_dir, exist_ok=True)
    ref = os.path.join(REPO, "oracle", "_ref")
    cases = {}
    for name, argv in CLI_BN.items():
        r = subprocess.run([os.path.join(ref, "bn")] + argv, cwd=MODELS, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, (name, r.returncode)
        cases[name] = {"tool": "bn", "argv": argv, "stdin": None, "stdout": r.stdout}
    for name, (argv, stdin) in CLI_MN.items():
        r = subprocess.run([os.path.join(ref, "mn")] + argv, cwd=MODELS, input=stdin, capture_output=True, text=True,
                           timeout=600)
        assert r.returncode == 0, (name, r.returncode)
        cases[name] = {"tool": "mn", "argv": argv, "stdin": stdin, "stdout": r.stdout}
    with open(os.path.join(HERE, "cli_golden.json"), "w") as f:
        json.dump(cases, f, indent=1)
    print("cli cases", len(cases))


# BN::query_ve (model.cpp:204-248): the reference's own asia query file plus
# random queries on alarm, each as the REPL's `query T | E` (bn.cpp:263, 347)
QUERY_CASES = [("asia.uai", "asia.markov.query", "mf"), ("asia.uai", "asia.markov.query", "given"),
               ("alarm.uai", "alarm.query", "mf")]


def query_golden():
    shutil.copyfile(os.path.join(REF_MODELS, "bayesnets", "asia.markov.query"), model_path("asia.markov.query"))
    rng = random.Random(2024)
    lines = []
    for _ in range(12):
        vs = rng.sample(range(37), rng.randint(1, 5))
        nt = rng.randint(1, min(2, len(vs)))
        t, e = vs[:nt], vs[nt:]
        lines.append("query " + ", ".join(map(str, t)) + ((" | " + ", ".join(map(str, e))) if e else ""))
    with open(model_path("alarm.query"), "w") as f:
        f.write("\n".join(lines) + "\nquit\n")
    cases = []
    for model, qf, h in QUERY_CASES:
        res = parse_factors(run("query", model_path(model), h, model_path(qf)))
        queries = [l for l in open(model_path(qf)) if l.startswith("query ")]
        cases.append({"model": model, "queries": qf, "heuristic": h, "lines": [q.strip() for q in queries],
                      "results": [res["Q%d" % i] for i in range(len(queries))]})
        print("query", model, qf, h, len(queries))
    with open(os.path.join(HERE, "query_golden.json"), "w") as f:
        json.dump({"cases": cases}, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1:] == ["query"]:
        query_golden()
    elif sys.argv[1:] == ["cli"]:
        cli_golden()
    elif sys.argv[1:] == ["config4"]:
        config4_golden()
    elif sys.argv[1:] == ["sp"]:
        sp_golden()
    elif sys.argv[1:] == ["corpus"]:
        corpus_golden()
    else:
        main()
        sp_golden()
        corpus_golden()
        config4_golden()
        cli_golden()
        query_golden()
