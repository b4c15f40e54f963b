"""GPU parity of the two-pass bucket-tree marginals (bnpp_marginals_tree).

The reference computes each marginal with its own VE (model.cpp:326-334); the
bucket tree computes all of them from one forward and one backward pass over
the partition's bucket tree, so its sums are associated differently: parity is
to rounding, not bit-exact.  Tolerances: fp64 1e-12 absolute against the
oracle's marginals and the golden vectors; fp32 1e-5 absolute (north star:
PR/MAR within 1e-6 relative on Z-scale quantities; marginals are in [0, 1]).
"""
import math
import os

import pytest

import bnpp
import refcpu
from bnpp import synth
from conftest import evidence_of, model_path

pytestmark = pytest.mark.gpu


def _close(a, b, tol):
    return all(abs(x - y) <= tol for x, y in zip(a, b)) and len(a) == len(b)


@pytest.mark.parametrize("dtype", [bnpp.F64, bnpp.F32])
def test_tree_marginals_vs_golden(ctx, golden_ve, dtype):
    tol = 1e-12 if dtype == bnpp.F64 else 1e-5
    for case in golden_ve["mar"]:
        m = bnpp.Model.load(model_path(case["model"]))
        ev = evidence_of(case["evidence"])
        marg, _ = bnpp.marginals_tree(ctx, m, ev, case["heuristic"], dtype)
        for t, ref in case["marginals"].items():
            t = int(t)
            if not ref["scope"]:                          # evidence variable: one-hot
                assert marg[t][ev[t]] == 1.0 and sum(marg[t]) == 1.0
                continue
            assert _close(marg[t], ref["values"], tol), (case["model"], t, marg[t], ref["values"])


@pytest.mark.parametrize("name,evid", [("alarm.uai", "alarm.uai.evid"), ("network.uai", "network.uai.evid"),
                                       ("grid3x3.uai", "grid3x3-MAR.uai.evid"), ("ising6x6.uai", None)])
def test_tree_matches_oracle_per_target(ctx, name, evid):
    m = bnpp.Model.load(model_path(name))
    ev = bnpp.load_evidence(model_path(evid)) if evid else {}
    rm, _ = refcpu.Model.load(model_path(name)).marginals(ev, "mf")
    marg, _ = bnpp.marginals_tree(ctx, m, ev, "mf", bnpp.F64)
    for t in range(m.n_vars):
        if t in ev:
            assert marg[t] == [1.0 if s == ev[t] else 0.0 for s in range(m.cards[t])]
        else:
            assert _close(marg[t], rm[t], 1e-12), (name, t, marg[t], rm[t])


@pytest.mark.parametrize("spec", [("potts", 5, 5, 3), ("ising", 9, 7, 2), ("noisy_or", 0, 0, 2)])
def test_tree_matches_per_target_engine(ctx, tmp_path, spec):
    """Synthetic models (Potts k=3, a non-square Ising grid, a noisy-OR BN with
    evidence on the findings): tree == per-target VE on the device."""
    kind, r, c, _ = spec
    if kind == "potts":
        md = synth.potts_grid(r, c, k=3, seed=5)
        ev = {}
    elif kind == "ising":
        md = synth.ising_grid(r, c, seed=6)
        ev = {0: 1, r * c - 1: 0, 17: 1}
    else:
        md = synth.noisy_or_bn(14, 18, 3, seed=7)
        ev = {v: v % 2 for v in range(14, 14 + 18, 2)}
    m = bnpp.Model.from_dict(md)
    want, _ = bnpp.marginals(ctx, m, ev, "mf", bnpp.F64)
    got, _ = bnpp.marginals_tree(ctx, m, ev, "mf", bnpp.F64)
    for t in range(m.n_vars):
        assert _close(got[t], want[t], 1e-12), (spec, t, got[t], want[t])
    got32, _ = bnpp.marginals_tree(ctx, m, ev, "mf", bnpp.F32)
    for t in range(m.n_vars):
        assert _close(got32[t], want[t], 1e-5), (spec, t, got32[t], want[t])


def test_tree_explicit_order_and_target_subset(ctx):
    """A column-sweep order (a chain-shaped bucket tree) and a subset of targets
    in caller order."""
    m = bnpp.Model.from_dict(synth.ising_grid(8, 12, seed=8))
    col = [r * 12 + c for c in range(12) for r in range(8)]
    want, _ = bnpp.marginals(ctx, m, {}, "mf", bnpp.F64)
    targets = [95, 0, 40, 41, 7]
    got, _ = bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F64, targets=targets, order=col)
    assert list(got) == targets
    for t in targets:
        assert _close(got[t], want[t], 1e-12), (t, got[t], want[t])


def test_tree_20x20_consistent_with_conditioned_partitions(ctx):
    """Beyond the per-target path's reach in a test budget: marginals of a
    20x20 grid (column-sweep order, width 20) match Z(x_t = s) / Z."""
    m = bnpp.Model.from_dict(synth.ising_grid(20, 20, seed=9))
    col = [r * 20 + c for c in range(20) for r in range(20)]
    marg, _ = bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F64, order=col)
    for t, p in marg.items():
        assert abs(sum(p) - 1.0) < 1e-12
    lz = bnpp.partition(ctx, m, {}, "mf", bnpp.F64, order=col)[0]
    for t in (0, 210, 399):
        for s in range(2):
            lzs = bnpp.partition(ctx, m, {t: s}, "mf", bnpp.F64, order=col)[0]
            assert abs(10 ** (lzs - lz) - marg[t][s]) < 1e-11, (t, s)


def test_tree_32x32_full_size_consistent_with_conditioned_partitions():
    """BASELINE config 3 at its full size (the bench's MAR instance): 32x32
    Ising grid, column-sweep order (width 32), fp32 -- 2^32-entry messages
    (16 GiB), the checkpointed chain schedule, split runs of 8.  The reference
    cannot run it, so parity is through size-independent properties: every
    marginal sums to 1, and P(x_t = s) = Z(x_t = s) / Z from conditioned
    partitions (north-star tolerance 1e-6), and every marginal agrees with the
    fp64 MAR to 1e-6.  Own context, closed at the end, so its ~275 GB arena
    does not stay cached beside the session context."""
    c = bnpp.Context(0)
    try:
        m = bnpp.Model.from_dict(synth.ising_grid(32, 32, seed=0))
        col = [r * 32 + cc for cc in range(32) for r in range(32)]
        marg, _ = bnpp.marginals_tree(c, m, {}, "mf", bnpp.F32, order=col)
        assert len(marg) == 1024
        for t, p in marg.items():
            assert len(p) == 2 and min(p) >= 0.0 and abs(sum(p) - 1.0) < 1e-6, (t, p)
        lz = bnpp.partition(c, m, {}, "mf", bnpp.F32, order=col)[0]
        for t in (0, 527):
            lz0 = bnpp.partition(c, m, {t: 0}, "mf", bnpp.F32, order=col)[0]
            assert abs(10 ** (lz0 - lz) - marg[t][0]) < 1e-6, (t, 10 ** (lz0 - lz), marg[t])
        # every marginal against the same MAR in fp64 (the reference's
        # precision): another plan (32-GiB messages, five checkpoint slots,
        # separate belief passes) and other kernels -- 1e-6 over all 2,048
        # entries; fp64's own Z-ratio check at 1e-11
        m64, _ = bnpp.marginals_tree(c, m, {}, "mf", bnpp.F64, order=col)
        diff = max(abs(a - b) for t in range(1024) for a, b in zip(marg[t], m64[t]))
        assert diff < 1e-6, diff
        lz64 = bnpp.partition(c, m, {}, "mf", bnpp.F64, order=col)[0]
        lz0 = bnpp.partition(c, m, {1023: 0}, "mf", bnpp.F64, order=col)[0]
        assert abs(10 ** (lz0 - lz64) - m64[1023][0]) < 1e-11
    finally:
        c.close()


def test_tree_memory_budget_is_enforced(ctx):
    m = bnpp.Model.from_dict(synth.ising_grid(10, 10, seed=0))
    os.environ["BNPP_MEM_BUDGET_GB"] = "1e-7"
    try:
        with pytest.raises(bnpp.BnppError) as e:
            bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F64)
        assert e.value.status == bnpp.ERR_OOM
    finally:
        del os.environ["BNPP_MEM_BUDGET_GB"]


def test_tree_job_relaunch(ctx):
    m = bnpp.Model.from_dict(synth.ising_grid(7, 7, seed=1))
    job = bnpp.Job(ctx, m, "mar_tree", heuristic="mf", dtype=bnpp.F64)
    job.launch()
    a = job.results()
    job.launch()
    job.launch()
    assert job.results() == a
    job.close()


@pytest.mark.parametrize("slots", [1, 2, 3, 7, 64])
def test_tree_chain_checkpointed_matches(ctx, slots):
    """Chain-shaped bucket tree (column sweep) with forward messages recomputed
    from `slots` checkpoints (binomial checkpointing; 1 slot degenerates to
    quadratic recomputation): same marginals as the per-target engine."""
    m = bnpp.Model.from_dict(synth.ising_grid(6, 9, seed=11))
    col = [r * 9 + c for c in range(9) for r in range(6)]
    ev = {13: 1}
    want, _ = bnpp.marginals(ctx, m, ev, "mf", bnpp.F64)
    os.environ["BNPP_TREE_SLOTS"] = str(slots)
    try:
        got, _ = bnpp.marginals_tree(ctx, m, ev, "mf", bnpp.F64, order=col)
        got32, _ = bnpp.marginals_tree(ctx, m, ev, "mf", bnpp.F32, order=col)
    finally:
        del os.environ["BNPP_TREE_SLOTS"]
    for t in range(m.n_vars):
        assert _close(got[t], want[t], 1e-12), (slots, t, got[t], want[t])
        assert _close(got32[t], want[t], 1e-5), (slots, t, got32[t], want[t])


def test_tree_chain_mode_rejects_non_chain(ctx):
    m = bnpp.Model.load(model_path("alarm.uai"))
    os.environ["BNPP_TREE_SLOTS"] = "4"
    try:
        with pytest.raises(bnpp.BnppError) as e:
            bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F64)
        assert e.value.status == bnpp.ERR_UNSUPPORTED
    finally:
        del os.environ["BNPP_TREE_SLOTS"]


@pytest.mark.parametrize("n_parts", [2, 3, 5])
def test_tree_parts_sum_to_whole(ctx, n_parts):
    """bnpp_marginals_tree_part: each part's owned marginals equal the whole
    tree's, and the parts cover every target once (chain segments with the
    forward prefix streamed and the backward messages run down to the segment)."""
    m = bnpp.Model.from_dict(synth.ising_grid(7, 11, seed=12))
    col = [r * 11 + c for c in range(11) for r in range(7)]
    ev = {20: 0}
    want, _ = bnpp.marginals(ctx, m, ev, "mf", bnpp.F64)
    seen = []
    for part in range(n_parts):
        got, _ = bnpp.marginals_tree(ctx, m, ev, "mf", bnpp.F64, order=col, part=part, n_parts=n_parts)
        seen += list(got)
        for t, p in got.items():
            assert _close(p, want[t], 1e-12), (part, t, p, want[t])
    assert sorted(seen) == list(range(m.n_vars))


@pytest.mark.parametrize("dtype", [bnpp.F64, bnpp.F32])
def test_tree_chain_fused_runs_identical_to_unfused(ctx, dtype):
    """Fused sweep runs (chain.cuh: F buckets per pass, intermediate messages in
    registers) perform each bucket's arithmetic in the reference's order and
    differ from the one-bucket-per-launch run only by exact powers of two, so
    the marginals are bit-identical (fp64 and fp32)."""
    m = bnpp.Model.from_dict(synth.ising_grid(10, 13, seed=5))
    col = [r * 13 + c for c in range(13) for r in range(10)]
    ev = {31: 1, 77: 0}
    os.environ["BNPP_TREE_SLOTS"] = "3"
    try:
        fused, _ = bnpp.marginals_tree(ctx, m, ev, "mf", dtype, order=col)
        os.environ["BNPP_NO_CHAIN"] = "1"
        plain, _ = bnpp.marginals_tree(ctx, m, ev, "mf", dtype, order=col)
    finally:
        del os.environ["BNPP_TREE_SLOTS"]
        os.environ.pop("BNPP_NO_CHAIN", None)
    assert fused == plain
    want, _ = bnpp.marginals(ctx, m, ev, "mf", bnpp.F64)
    tol = 1e-12 if dtype == bnpp.F64 else 1e-5
    for t in range(m.n_vars):
        assert _close(fused[t], want[t], tol), (t, fused[t], want[t])


@pytest.mark.parametrize("dtype", [bnpp.F64, bnpp.F32])
def test_tree_chain_fused_potts4(ctx, dtype):
    """4-state Potts column sweep: chain runs over K = 4 slots (16-entry register
    tables), identical to one bucket per launch and to the per-target engine."""
    m = bnpp.Model.from_dict(synth.potts_grid(5, 7, k=4, seed=3))
    col = [r * 7 + c for c in range(7) for r in range(5)]
    ev = {9: 2}
    os.environ["BNPP_TREE_SLOTS"] = "2"
    try:
        fused, _ = bnpp.marginals_tree(ctx, m, ev, "mf", dtype, order=col)
        os.environ["BNPP_NO_CHAIN"] = "1"
        plain, _ = bnpp.marginals_tree(ctx, m, ev, "mf", dtype, order=col)
    finally:
        del os.environ["BNPP_TREE_SLOTS"]
        os.environ.pop("BNPP_NO_CHAIN", None)
    assert fused == plain
    want, _ = bnpp.marginals(ctx, m, ev, "mf", bnpp.F64)
    tol = 1e-12 if dtype == bnpp.F64 else 1e-5
    for t in range(m.n_vars):
        assert _close(fused[t], want[t], tol), (t, fused[t], want[t])


@pytest.mark.parametrize("shape", [(2, 9, 14), (4, 5, 8)])
def test_partition_fused_sweep_matches_oracle(ctx, shape):
    """plan_ve with fused sweep runs (column order): log10 Z bit-identical to
    one bucket per launch in fp64, and equal to the oracle's Z to 1e-12."""
    import refcpu
    k, r, c = shape
    d = synth.ising_grid(r, c, seed=4) if k == 2 else synth.potts_grid(r, c, k=k, seed=4)
    m = bnpp.Model.from_dict(d)
    col = [i * c + j for j in range(c) for i in range(r)]
    lz, z, _ = bnpp.partition(ctx, m, {}, "mf", bnpp.F64, order=col)
    os.environ["BNPP_NO_CHAIN"] = "1"
    try:
        lz_plain, _, _ = bnpp.partition(ctx, m, {}, "mf", bnpp.F64, order=col)
        lz32_plain, _, _ = bnpp.partition(ctx, m, {}, "mf", bnpp.F32, order=col)
    finally:
        del os.environ["BNPP_NO_CHAIN"]
    lz32, _, _ = bnpp.partition(ctx, m, {}, "mf", bnpp.F32, order=col)
    assert lz == lz_plain and lz32 == lz32_plain
    rz, _ = refcpu.Model.from_dict(d).partition({}, "mf")      # oracle: min-fill order, fp64
    assert abs(lz - math.log10(rz)) < 1e-12 * abs(lz)
    assert abs(lz32 - lz) < 1e-6 * abs(lz)


@pytest.mark.parametrize("spec", [(2, 14, 5), (4, 7, 4)])
def test_summing_runs_identical_to_unfused(ctx, spec):
    """The last column of a tall sweep only sums variables out (kChainSum runs):
    partition and tree marginals bit-identical to one bucket per launch."""
    k, r, c = spec
    d = synth.ising_grid(r, c, seed=8) if k == 2 else synth.potts_grid(r, c, k=k, seed=8)
    m = bnpp.Model.from_dict(d)
    col = [i * c + j for j in range(c) for i in range(r)]
    res = {}
    for nc in ("0", "1"):
        os.environ["BNPP_NO_CHAIN"] = nc
        os.environ["BNPP_TREE_SLOTS"] = "3"
        try:
            res[nc] = [bnpp.partition(ctx, m, {}, "mf", dt, order=col)[0] for dt in (bnpp.F64, bnpp.F32)]
            res[nc] += [bnpp.marginals_tree(ctx, m, {}, "mf", dt, order=col)[0] for dt in (bnpp.F64, bnpp.F32)]
        finally:
            del os.environ["BNPP_NO_CHAIN"]
            del os.environ["BNPP_TREE_SLOTS"]
    assert res["0"] == res["1"]


@pytest.mark.parametrize("spec", [(2, 16, 5), (4, 8, 4)])
def test_short_forward_runs_vector_form(ctx, spec):
    """Short forward runs (2..4 buckets) take the V-wide forward form
    (kChainFwdV, several rest entries per thread): partition and tree marginals
    bit-identical to the one-entry form and to one bucket per launch."""
    k, r, c = spec
    d = synth.ising_grid(r, c, seed=11) if k == 2 else synth.potts_grid(r, c, k=k, seed=11)
    m = bnpp.Model.from_dict(d)
    col = [i * c + j for j in range(c) for i in range(r)]
    knobs = [{"BNPP_CHAIN_RUN_MAX": str(rm)} for rm in (2, 3, 4)]
    knobs += [dict(kn, BNPP_NO_CHAIN_FWDV="1") for kn in knobs] + [{"BNPP_NO_CHAIN": "1"}]
    res = []
    for kn in knobs:
        os.environ.update(kn)
        os.environ["BNPP_TREE_SLOTS"] = "3"
        try:
            out = [bnpp.partition(ctx, m, {}, "mf", dt, order=col)[0] for dt in (bnpp.F64, bnpp.F32)]
            out += [bnpp.marginals_tree(ctx, m, {}, "mf", dt, order=col)[0] for dt in (bnpp.F64, bnpp.F32)]
            res.append(out)
        finally:
            for key in list(kn) + ["BNPP_TREE_SLOTS"]:
                del os.environ[key]
    for out in res[1:]:
        assert out == res[0]


@pytest.mark.parametrize("spec", [(16, 6, None), (18, 5, {3: 1, 40: 0}), (17, 4, None), (20, 3, {7: 0})])
def test_split_runs_identical_to_unfused(ctx, capfd, spec):
    """Binary fp32 sweeps tall enough for the split chain form (chainsplit.cuh:
    runs of 5..8 buckets, the 2^F table of a rest entry over 2^(F-4) waves):
    partition and tree marginals bit-identical to the one-thread runs of <= 6
    buckets and to one bucket per launch; the plan holds split runs with dense
    addressing (forms 7, 8) and, with BNPP_NO_DENSE, with the general one
    (forms 5, 6) -- both bit-identical (the split runs fold their rescale
    into the last G table)."""
    r, c, ev = spec
    ev = ev or {}
    m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=13))
    col = [i * c + j for j in range(c) for i in range(r)]
    knobs = [{"BNPP_DEBUG_CHAIN": "1"}, {"BNPP_DEBUG_CHAIN": "1", "BNPP_NO_DENSE": "1"}, {"BNPP_SPLIT_MIN_F": "7"},
             {"BNPP_NO_SPLIT": "1"}, {"BNPP_NO_SPLIT": "1", "BNPP_CHAIN_RUN_MAX": "6"}, {"BNPP_NO_CHAIN": "1"}]
    res = []
    for kn in knobs:
        os.environ.update(kn)
        os.environ["BNPP_TREE_SLOTS"] = "3"
        capfd.readouterr()
        try:
            # evidence in the partition only (it can branch the bucket tree, and
            # BNPP_TREE_SLOTS forces the checkpointed chain plan)
            out = [bnpp.partition(ctx, m, ev, "mf", bnpp.F32, order=col)[0],
                   bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F32, order=col)[0]]
            res.append(out)
        finally:
            for key in list(kn) + ["BNPP_TREE_SLOTS"]:
                del os.environ[key]
        if "BNPP_DEBUG_CHAIN" in kn:
            err = capfd.readouterr().err
            forms = (5, 6) if "BNPP_NO_DENSE" in kn else (7, 8)
            assert any("run form %d K=2 F=8" % f in err for f in forms), err[-2000:]
    for out in res[1:]:
        assert out == res[0]
    want, _ = bnpp.marginals(ctx, m, {}, "mf", bnpp.F64)
    for t in range(m.n_vars):
        assert _close(res[0][1][t], want[t], 1e-5), (t, res[0][1][t], want[t])


@pytest.mark.parametrize("spec", [(16, 6, None, None), (18, 5, {3: 1, 40: 0}, None), (17, 4, None, 11)])
def test_split_runs_fp64_identical_to_unfused(ctx, capfd, spec):
    """fp64 split runs (chainsplit.cuh with T = double: runs of 5..8 buckets,
    16 entries per lane, scalar fp64 arithmetic in the reference's order; runs
    of 8 on the aliased LDS layout, split_alias): partition and tree marginals
    bit-identical to the one-thread runs, to one bucket per launch, dense and
    general addressing alike; the last spec has peaked potentials (every fused
    run rescales by 2^-50 or more).  The plan holds F = 8 split runs (forms 7,
    8 dense; 5, 6 general)."""
    r, c, ev, log2_eps = spec
    ev = ev or {}
    d = synth.ising_grid(r, c, seed=13) if log2_eps is None else synth.peaked_grid(r, c, log2_eps=log2_eps, seed=5)
    m = bnpp.Model.from_dict(d)
    col = [i * c + j for j in range(c) for i in range(r)]
    knobs = [{"BNPP_DEBUG_CHAIN": "1"}, {"BNPP_DEBUG_CHAIN": "1", "BNPP_NO_DENSE": "1"}, {"BNPP_NO_SPLIT": "1"},
             {"BNPP_NO_CHAIN": "1"}]
    res = []
    for kn in knobs:
        os.environ.update(kn)
        os.environ["BNPP_TREE_SLOTS"] = "3"
        capfd.readouterr()
        try:
            out = [bnpp.partition(ctx, m, ev, "mf", bnpp.F64, order=col)[0],
                   bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F64, order=col)[0]]
            res.append(out)
        finally:
            for key in list(kn) + ["BNPP_TREE_SLOTS"]:
                del os.environ[key]
        if "BNPP_DEBUG_CHAIN" in kn:
            err = capfd.readouterr().err
            forms = (5, 6) if "BNPP_NO_DENSE" in kn else (7, 8)
            assert any("run form %d K=2 F=8" % f in err for f in forms), err[-2000:]
    for out in res[1:]:
        assert out == res[0]
    want, _ = bnpp.marginals(ctx, m, {}, "mf", bnpp.F64)
    for t in range(m.n_vars):
        assert _close(res[0][1][t], want[t], 1e-12), (t, res[0][1][t], want[t])
    rz, _ = refcpu.Model.from_dict(d).partition(ev, "mf")
    assert abs(res[0][0] - math.log10(rz)) <= 1e-12 * abs(math.log10(rz)), (res[0][0], math.log10(rz))


def _bucket_max_log2(d, rows, cols):
    """max over x of the product of the column-sweep bucket of each variable
    above the last row (unary, right pair, down pair), as log2"""
    vals = {tuple(s): v for s, v in zip(d["scopes"], d["values"])}
    worst = -1e9
    for r in range(rows - 1):
        for c in range(cols):
            v = r * cols + c
            un, dn = vals[(v,)], vals[(v, v + cols)]
            rt = vals[(v, v + 1)] if c + 1 < cols else [1.0] * 4
            best = max(un[x] * dn[2 * x + y] * rt[2 * x + z] for x in range(2) for y in range(2) for z in range(2))
            worst = max(worst, math.log2(best))
    return worst


@pytest.mark.parametrize("rows,cols,log2_eps", [(16, 4, 10), (18, 3, 12), (17, 3, 13)])
def test_split_runs_peaked_potentials(ctx, capfd, rows, cols, log2_eps):
    """Potentials whose bucket products peak far below 1 (synth.peaked_grid:
    every bucket above the last row has max <= 2^-log2_eps, so a fused run of
    F >= 5 buckets carries a rescale 2^-sum(e) with |sum(e)| >= 5 (log2_eps - 1)
    = 45..95 -- outside the +-32 that round 3's last-table fold covered, where
    it left the scale unapplied and the values drifted toward underflow).  The
    rescale is now folded per bucket (chain.cuh chain_fold), so split runs
    (dense and general addressing, F >= 7), one-thread runs (F <= 6) and one
    bucket per launch give bit-identical fp32 partitions and tree marginals,
    and log10 Z agrees with the fp64 oracle (reference arithmetic, factor.cpp:
    131-143, 199-205; no scaling) to fp32 rounding."""
    d = synth.peaked_grid(rows, cols, log2_eps=log2_eps, seed=5)
    assert _bucket_max_log2(d, rows, cols) <= -log2_eps + 1e-9
    m = bnpp.Model.from_dict(d)
    col = [i * cols + j for j in range(cols) for i in range(rows)]
    knobs = [{"BNPP_DEBUG_CHAIN": "1"}, {"BNPP_DEBUG_CHAIN": "1", "BNPP_NO_DENSE": "1"}, {"BNPP_SPLIT_MIN_F": "7"},
             {"BNPP_NO_SPLIT": "1"}, {"BNPP_NO_SPLIT": "1", "BNPP_CHAIN_RUN_MAX": "6"}, {"BNPP_NO_CHAIN": "1"}]
    res = []
    for kn in knobs:
        os.environ.update(kn)
        os.environ["BNPP_TREE_SLOTS"] = "3"
        capfd.readouterr()
        try:
            out = [bnpp.partition(ctx, m, {}, "mf", bnpp.F32, order=col)[0],
                   bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F32, order=col)[0]]
            res.append(out)
        finally:
            for key in list(kn) + ["BNPP_TREE_SLOTS"]:
                del os.environ[key]
        if "BNPP_DEBUG_CHAIN" in kn:
            err = capfd.readouterr().err
            forms = (5, 6) if "BNPP_NO_DENSE" in kn else (7, 8)
            assert any("run form %d K=2 F=8" % f in err for f in forms), err[-2000:]
    for out in res[1:]:
        assert out == res[0]
    rz, _ = refcpu.Model.from_dict(d).partition({}, "mf")
    assert rz > 0.0
    lz_ref = math.log10(rz)
    assert abs(res[0][0] - lz_ref) <= 1e-6 * abs(lz_ref), (res[0][0], lz_ref)
    # fp64: min-fill plan bit-exact vs the oracle, the column sweep to 1e-12
    lz64, z64, _ = bnpp.partition(ctx, m, {}, "mf", bnpp.F64)
    assert z64 == rz
    lz64c = bnpp.partition(ctx, m, {}, "mf", bnpp.F64, order=col)[0]
    assert abs(lz64c - lz_ref) <= 1e-12 * abs(lz_ref)
    want, _ = bnpp.marginals(ctx, m, {}, "mf", bnpp.F64)
    for t in range(m.n_vars):
        assert _close(res[0][1][t], want[t], 1e-5), (t, res[0][1][t], want[t])


@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_slab_outer_dims_identical_to_stream(ctx, capfd, dt):
    """A column sweep's first buckets multiply a growing message by factors
    over new variables: [S slab][2][2] outputs whose big input is contiguous
    along the slab dim and constant or strided along the slower ones.  They run
    as slab tiles with the slower dims enumerated per block (outer=4), bit-
    identical to the stream kernel (BNPP_NO_SLAB_OUTER) and to one bucket per
    launch without either (BNPP_NO_SLAB + BNPP_NO_CHAIN): same product order
    (factor.cpp:131-143), same rescale.  fp64 tree marginals also match the
    per-target engine to 1e-12."""
    r = c = 16
    m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=41))
    col = [i * c + j for j in range(c) for i in range(r)]
    d = bnpp.F64 if dt == "f64" else bnpp.F32
    knobs = [{"BNPP_DUMP_PLAN": "1"}, {"BNPP_NO_SLAB_OUTER": "1"}, {"BNPP_NO_SLAB": "1", "BNPP_NO_CHAIN": "1"}]
    res = []
    for kn in knobs:
        os.environ.update(kn)
        capfd.readouterr()
        try:
            res.append([bnpp.partition(ctx, m, {}, "mf", d, order=col)[0],
                        bnpp.marginals_tree(ctx, m, {}, "mf", d, order=col)[0]])
        finally:
            for key in kn:
                del os.environ[key]
        if "BNPP_DUMP_PLAN" in kn:
            outer = [ln for ln in capfd.readouterr().err.splitlines() if " outer=" in ln]
            assert len(outer) >= 2, len(outer)
    for out in res[1:]:
        assert out == res[0]
    if dt == "f64":
        want, _ = bnpp.marginals(ctx, m, {}, "mf", bnpp.F64)
        for t in range(m.n_vars):
            assert _close(res[0][1][t], want[t], 1e-12), (t, res[0][1][t], want[t])


def _two_grids(a, b):
    n = len(a["cards"])
    return {"type": "MARKOV", "cards": a["cards"] + b["cards"],
            "scopes": a["scopes"] + [[v + n for v in s] for s in b["scopes"]], "values": a["values"] + b["values"]}


@pytest.mark.parametrize("model,dt", [("ising", "f32"), ("peaked", "f32"), ("two", "f32"), ("ising", "f64"),
                                      ("peaked", "f64")])
def test_fused_beliefs_identical_to_belief_passes(ctx, capfd, model, dt):
    """Deliveries whose belief sums the slots of the backward run that made
    its message (kChainBel: 16x6 column sweeps with 2^8-entry kept sets, so a
    belief sums 8 binary variables) are formed inside that run -- it also
    reads the forward message and adds lam * pi over its 256 slot
    combinations in slab order -- instead of a separate pass over lam and pi.
    The belief is stored unscaled (its exp2 carries the inputs'), so the tree
    marginals are bit-identical to the separate belief passes
    (BNPP_NO_BEL_FUSE), to one-thread runs and to one bucket per launch, and
    within fp32 rounding of the fp64 per-target engine; peaked potentials
    (every bucket product <= 2^-10) and two disconnected grids included.
    fp64: split runs of 7 buckets, 2^9-entry kept sets (a belief sums 7
    variables), the fp64 belief kernel; within 1e-12 of the per-target engine."""
    dtype = bnpp.F32 if dt == "f32" else bnpp.F64
    keep = "8" if dt == "f32" else "9"
    if model == "ising":
        d = synth.ising_grid(16, 6, seed=31)
    elif model == "peaked":
        d = synth.peaked_grid(16, 6, log2_eps=10, seed=32)
    else:
        d = _two_grids(synth.ising_grid(16, 6, seed=33), synth.ising_grid(16, 6, seed=34))
    m = bnpp.Model.from_dict(d)
    col = [i * 6 + j for j in range(6) for i in range(16)]
    order = col if model != "two" else col + [v + 96 for v in col]
    knobs = [{"BNPP_DUMP_PLAN": "1"}, {"BNPP_NO_BEL_FUSE": "1"}, {"BNPP_NO_SPLIT": "1"}, {"BNPP_NO_CHAIN": "1"}]
    res = []
    for kn in knobs:
        os.environ.update(kn)
        os.environ.update({"BNPP_KEEP_LOG2": keep, "BNPP_TREE_SLOTS": "3"})
        capfd.readouterr()
        try:
            res.append(bnpp.marginals_tree(ctx, m, {}, "mf", dtype, order=order)[0])
        finally:
            for key in list(kn) + ["BNPP_KEEP_LOG2", "BNPP_TREE_SLOTS"]:
                del os.environ[key]
        if "BNPP_DUMP_PLAN" in kn:
            fused = [ln for ln in capfd.readouterr().err.splitlines() if " belief: " in ln]
            assert len(fused) >= (8 if model != "two" else 16) - (1 if dt == "f64" else 0), len(fused)
    for out in res[1:]:
        assert out == res[0]
    want, _ = bnpp.marginals(ctx, m, {}, "mf", bnpp.F64)
    tol = 1e-5 if dt == "f32" else 1e-12
    for t in range(m.n_vars):
        assert _close(res[0][t], want[t], tol), (t, res[0][t], want[t])


@pytest.mark.parametrize("n_parts", [2, 3])
def test_fused_beliefs_in_tree_parts(ctx, capfd, n_parts):
    """The segment-owned parts (bnpp_marginals_tree_part, the N-GPU MAR) fuse
    the beliefs of their own deliveries the same way: every part's marginals
    bit-identical with and without the fusion, the parts covering every target
    once, within fp32 rounding of the fp64 per-target engine."""
    m = bnpp.Model.from_dict(synth.ising_grid(16, 6, seed=35))
    col = [i * 6 + j for j in range(6) for i in range(16)]
    want, _ = bnpp.marginals(ctx, m, {}, "mf", bnpp.F64)
    got = {}
    n_fused = 0
    for kn in ({"BNPP_DUMP_PLAN": "1"}, {"BNPP_NO_BEL_FUSE": "1"}):
        os.environ.update(kn)
        os.environ.update({"BNPP_KEEP_LOG2": "8", "BNPP_TREE_SLOTS": "3"})
        capfd.readouterr()
        try:
            parts = [bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F32, order=col, part=p, n_parts=n_parts)[0]
                     for p in range(n_parts)]
        finally:
            for key in list(kn) + ["BNPP_KEEP_LOG2", "BNPP_TREE_SLOTS"]:
                del os.environ[key]
        if "BNPP_DUMP_PLAN" in kn:
            n_fused = sum(" belief: " in ln for ln in capfd.readouterr().err.splitlines())
        got[tuple(kn)] = parts
    assert n_fused >= 4, n_fused
    a, b = got[("BNPP_DUMP_PLAN",)], got[("BNPP_NO_BEL_FUSE",)]
    assert a == b
    seen = [t for part in a for t in part]
    assert sorted(seen) == list(range(m.n_vars))
    for part in a:
        for t, p in part.items():
            assert _close(p, want[t], 1e-5), (t, p, want[t])


@pytest.mark.parametrize("keep,slow,rows", [(3, 13, 12), (5, 13, 12), (7, 2, 12), (9, 4, 12), (13, 13, 14)])
def test_tree_chain_kept_sets_match(ctx, keep, slow, rows):
    """Deliveries from kept sets smaller than the separators (the 32x32 path:
    slow variables summed in one composite pass, the others reduced from the
    kept table; targets never kept get their own reduction), forced on a
    12x10 column sweep by shrinking the kept / slow limits (14x10 with 2^13
    kept entries: kept tables reduced hierarchically, reduce_many): same
    marginals as the per-target engine."""
    m = bnpp.Model.from_dict(synth.ising_grid(rows, 10, seed=12))
    col = [r * 10 + c for c in range(10) for r in range(rows)]
    want, _ = bnpp.marginals(ctx, m, {}, "mf", bnpp.F64)
    os.environ.update({"BNPP_KEEP_LOG2": str(keep), "BNPP_SLOW_LOG2": str(slow), "BNPP_TREE_SLOTS": "3"})
    try:
        got, _ = bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F64, order=col)
        got32, _ = bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F32, order=col)
    finally:
        for k in ("BNPP_KEEP_LOG2", "BNPP_SLOW_LOG2", "BNPP_TREE_SLOTS"):
            os.environ.pop(k, None)
    for t in range(m.n_vars):
        assert _close(got[t], want[t], 1e-12), (keep, slow, t, got[t], want[t])
        assert _close(got32[t], want[t], 1e-5), (keep, slow, t, got32[t], want[t])


def test_split_runs_of_two_components_share_launches(ctx, capfd):
    """Two disconnected 18x5 grids: their sweeps' split runs land on the same
    levels, so a launch carries several run descriptors (the kernel's
    multi-bucket path: per-tile bucket lookup, G tables restaged at bucket
    changes).  log10 Z bit-identical to one-thread runs and to one bucket per
    launch, and equal to the sum of the components' log10 Z."""
    a, b = synth.ising_grid(18, 5, seed=21), synth.ising_grid(18, 5, seed=22)
    n = len(a["cards"])
    md = {"type": "MARKOV", "cards": a["cards"] + b["cards"],
          "scopes": a["scopes"] + [[v + n for v in s] for s in b["scopes"]], "values": a["values"] + b["values"]}
    m = bnpp.Model.from_dict(md)
    col = [i * 5 + j for j in range(5) for i in range(18)]
    order = col + [v + n for v in col]
    res = []
    for kn in ({"BNPP_DUMP_PLAN": "1"}, {"BNPP_NO_SPLIT": "1"}, {"BNPP_NO_CHAIN": "1"}):
        os.environ.update(kn)
        capfd.readouterr()
        try:
            res.append(bnpp.partition(ctx, m, {}, "mf", bnpp.F32, order=order)[0])
        finally:
            for key in kn:
                del os.environ[key]
        if "BNPP_DUMP_PLAN" in kn:
            runs = [ln.split()[0] for ln in capfd.readouterr().err.splitlines() if " chain F=8 " in ln]
            assert runs and max(runs.count(lv) for lv in runs) >= 2, runs
    assert res[1] == res[0] and res[2] == res[0]
    ma, mb = bnpp.Model.from_dict(a), bnpp.Model.from_dict(b)
    want = bnpp.partition(ctx, ma, {}, "mf", bnpp.F64, order=col)[0] + bnpp.partition(ctx, mb, {}, "mf", bnpp.F64, order=col)[0]
    assert abs(res[0] - want) <= 1e-6 * abs(want), (res[0], want)


@pytest.mark.parametrize("rows,cols,hop", [(12, 6, 3), (10, 5, 2)])
def test_runs_with_non_neighbour_g_fall_back_safely(ctx, rows, cols, hop):
    """A column sweep whose buckets also hold a factor to the variable `hop`
    rows below (G_j depends on slot j + hop, not a neighbouring one: ChainDep
    any).  Such runs cannot use the split forms; the planner falls back to the
    one-thread forms only where their own layout conditions hold (ADVICE r2:
    a backward fallback once skipped them), else to shorter runs.  Partition
    and tree marginals bit-identical across the chain variants, and within
    tolerance of the oracle's fp64 partition."""
    import random
    d = synth.ising_grid(rows, cols, seed=31)
    rng = random.Random(5)
    for c in range(cols):
        for r in range(rows - hop):
            j = rng.uniform(-0.5, 0.5)
            e, ne = round(math.exp(j), 6), round(math.exp(-j), 6)
            d["scopes"].append([r * cols + c, (r + hop) * cols + c])
            d["values"].append([e, ne, ne, e])
    m = bnpp.Model.from_dict(d)
    col = [i * cols + j for j in range(cols) for i in range(rows)]
    knobs = [{}, {"BNPP_NO_SPLIT": "1"}, {"BNPP_NO_DENSE": "1"}, {"BNPP_CHAIN_RUN_MAX": "5"}, {"BNPP_NO_CHAIN": "1"}]
    res = []
    for kn in knobs:
        os.environ.update(kn)
        os.environ["BNPP_TREE_SLOTS"] = "3"
        try:
            res.append([bnpp.partition(ctx, m, {}, "mf", dt, order=col)[0] for dt in (bnpp.F64, bnpp.F32)] +
                       [bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F32, order=col)[0]])
        finally:
            for key in list(kn) + ["BNPP_TREE_SLOTS"]:
                del os.environ[key]
    for out in res[1:]:
        assert out == res[0]
    assert abs(res[0][1] - res[0][0]) <= 1e-6 * abs(res[0][0])
    want, _ = bnpp.marginals(ctx, m, {}, "mf", bnpp.F64)
    for t in range(m.n_vars):
        assert _close(res[0][2][t], want[t], 1e-5), (t, res[0][2][t], want[t])


def test_split_runs_fp64_multi_run_levels(ctx, capfd):
    """A grid cut in two by a column of evidence sweeps both halves at once:
    the PR has levels holding two fp64 split runs of 8 (one launch, the
    multi-run kernel on the aliased LDS layout, chainsplit.cuh MODE 2).  Partition and tree
    marginals bit-identical to one-thread runs and to one bucket per launch;
    marginals equal per-target VE to 1e-12."""
    r, c = 16, 13
    d = synth.ising_grid(r, c, seed=13)
    m = bnpp.Model.from_dict(d)
    ev = {i * c + 6: i % 2 for i in range(r)}
    col = [i * c + j for j in range(c) for i in range(r)]
    # the PR plan holds levels with two runs of 8 (host-side planning dump)
    os.environ["BNPP_DUMP_PLAN"] = "1"
    capfd.readouterr()
    try:
        bnpp.plan_stats(m, 0, ev, "mf", dtype=bnpp.F64, order=col)
    finally:
        del os.environ["BNPP_DUMP_PLAN"]
    runs = {}
    for line in capfd.readouterr().err.splitlines():
        if " chain F=8 " in line:
            lvl = line.split()[0]
            runs[lvl] = runs.get(lvl, 0) + 1
    assert any(n >= 2 for n in runs.values()), runs
    res = []
    for kn in ({}, {"BNPP_NO_SPLIT": "1"}, {"BNPP_NO_CHAIN": "1"}):
        os.environ.update(kn)
        try:
            res.append([bnpp.partition(ctx, m, ev, "mf", bnpp.F64, order=col)[0],
                        bnpp.marginals_tree(ctx, m, ev, "mf", bnpp.F64, order=col)[0]])
        finally:
            for key in kn:
                del os.environ[key]
    for out in res[1:]:
        assert out == res[0]
    want, _ = bnpp.marginals(ctx, m, ev, "mf", bnpp.F64)
    for t in range(m.n_vars):
        assert _close(res[0][1][t], want[t], 1e-12), (t, res[0][1][t], want[t])
