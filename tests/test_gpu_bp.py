"""Loopy BP (`bn -sp`, BN::marginals with options["sum-product"],
model.cpp:313-317, 736-753; graph.cpp:256-403) on the device (bp.hip through
the C ABI bnpp_sum_product) against the reference's own outputs
(tests/golden/sp_golden.json, made by oracle/_ref/ref_harness) and, for
instances the golden set does not hold, against the oracle (refcpu.c).

Tolerance: the flooding schedule is the reference's; products run in a fixed
order where the reference walks unordered_maps, so marginals agree to
rounding: 1e-12 absolute (fp64), iteration counts exactly."""
import pytest

import bnpp
import refcpu
from bnpp import synth
from conftest import model_path

pytestmark = pytest.mark.gpu

TOL = 1e-12


class _env:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        import os
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *exc):
        import os
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _check(got, want, tag):
    assert set(got) == set(int(t) for t in want), tag
    for t, ref in want.items():
        g = got[int(t)]
        assert len(g) == len(ref), (tag, t)
        for a, b in zip(g, ref):
            assert abs(a - b) <= TOL, (tag, t, a, b)


def test_sum_product_matches_reference(ctx, golden_sp):
    """Every golden case: BNs (trees and loopy), Ising / Potts grids, a noisy-OR
    net, a 3x3 grid that does not converge within its cap, and max_iter = 0."""
    for case in golden_sp["cases"]:
        m = bnpp.Model.load(model_path(case["model"]))
        marg, it, _ = bnpp.sum_product(ctx, m, case["max_iter"], case["eps"])
        tag = (case["model"], case["max_iter"], case["eps"])
        assert it == case["iterations"], (tag, it)
        _check(marg, case["marginals"], tag)


@pytest.mark.parametrize("spec", [("ising", 20, 20, 1e-6), ("potts", 9, 11, 1e-4), ("noisyor", 60, 90, 1e-3)])
def test_sum_product_matches_oracle_larger(ctx, spec, tmp_path):
    """Loopy models with more edges than the workgroup has threads: same
    iterations and marginals as the oracle's restatement."""
    kind, a, b, eps = spec
    if kind == "ising":
        d = synth.ising_grid(a, b, seed=21)
    elif kind == "potts":
        d = synth.potts_grid(a, b, k=3, seed=21)
    else:
        d = synth.noisy_or_bn(a, b, 4, seed=21)
    path = str(tmp_path / "m.uai")
    synth.write_uai(d, path)
    want, want_it, _ = refcpu.Model.load(path).sum_product(10000, eps)
    marg, it, _ = bnpp.sum_product(ctx, bnpp.Model.load(path), 10000, eps)
    assert it == want_it
    _check(marg, {str(k): v for k, v in want.items()}, kind)


def test_sum_product_repeatable(ctx):
    """Two calls give identical bits (one workgroup, fixed order)."""
    m = bnpp.Model.load(model_path("alarm.uai"))
    r1 = bnpp.sum_product(ctx, m)
    r2 = bnpp.sum_product(ctx, m)
    assert r1[0] == r2[0] and r1[1] == r2[1]


@pytest.mark.parametrize("model", ["pathfinder.uai", "ising10x10.uai"])
def test_sum_product_global_messages_identical(ctx, model):
    """One-workgroup loop: messages in global memory (BNPP_BP_NO_LDS, the path
    of models with more than 4096 message entries) give the same bits as
    messages in LDS."""
    m = bnpp.Model.load(model_path(model))
    with _env(BNPP_BP_MODE="single"):
        lds = bnpp.sum_product(ctx, m, 10000, 1e-6)
        with _env(BNPP_BP_NO_LDS="1"):
            glb = bnpp.sum_product(ctx, m, 10000, 1e-6)
    assert lds[0] == glb[0] and lds[1] == glb[1]


# --- multi-workgroup flood (bp.hip bp_flood_*: one launch per phase and
# iteration, the choice for large models and for tables of 2^31+ entries) ---
@pytest.mark.parametrize("idx64", ["0", "1"])
def test_flood_matches_reference(ctx, golden_sp, idx64):
    """Every golden case on the multi-workgroup flood (BNPP_BP_MODE=multi),
    32-bit and forced 64-bit table indices: the reference's iteration counts
    exactly (including the 3x3 grid that runs to its cap and max_iter = 0),
    marginals within 1e-12."""
    kv = {"BNPP_BP_MODE": "multi"}
    if idx64 == "1":
        kv["BNPP_BP_IDX64"] = "1"
    with _env(**kv):
        for case in golden_sp["cases"]:
            m = bnpp.Model.load(model_path(case["model"]))
            marg, it, _ = bnpp.sum_product(ctx, m, case["max_iter"], case["eps"])
            tag = (case["model"], case["max_iter"], case["eps"], "multi", idx64)
            assert it == case["iterations"], (tag, it)
            _check(marg, case["marginals"], tag)


@pytest.mark.parametrize("spec", [("ising", 20, 20, 1e-6), ("potts", 9, 11, 1e-4), ("noisyor", 60, 90, 1e-3)])
def test_flood_matches_oracle_larger(ctx, spec, tmp_path):
    """The flood against the oracle on loopy models larger than one workgroup."""
    kind, a, b, eps = spec
    if kind == "ising":
        d = synth.ising_grid(a, b, seed=21)
    elif kind == "potts":
        d = synth.potts_grid(a, b, k=3, seed=21)
    else:
        d = synth.noisy_or_bn(a, b, 4, seed=21)
    path = str(tmp_path / "m.uai")
    synth.write_uai(d, path)
    want, want_it, _ = refcpu.Model.load(path).sum_product(10000, eps)
    with _env(BNPP_BP_MODE="multi"):
        marg, it, _ = bnpp.sum_product(ctx, bnpp.Model.load(path), 10000, eps)
    assert it == want_it
    _check(marg, {str(k): v for k, v in want.items()}, kind)


def test_flood_chosen_for_large_models_and_agrees_with_one_workgroup(ctx):
    """A 120x120 Ising grid is past the one-workgroup work bound, so the
    default call floods; forcing the one-workgroup loop gives the same
    iteration count and marginals within 1e-12; the flood is repeatable."""
    m = bnpp.Model.from_dict(synth.ising_grid(120, 120, seed=5))
    auto = bnpp.sum_product(ctx, m, 10000, 1e-6)
    with _env(BNPP_BP_MODE="multi"):
        multi = bnpp.sum_product(ctx, m, 10000, 1e-6)
    with _env(BNPP_BP_MODE="single"):
        single = bnpp.sum_product(ctx, m, 10000, 1e-6)
    assert auto[0] == multi[0] and auto[1] == multi[1]
    assert single[1] == multi[1]
    _check(multi[0], {str(k): v for k, v in single[0].items()}, "ising120")


def test_flood_table_beyond_2_31_entries(ctx):
    """One factor of 1291^3 = 2,151,685,171 entries (past the one-workgroup
    loop's 2^31 bound; the reference has no bound, graph.cpp:364-391): the
    table is u0 (x) u1 (x) u2 and each variable also has a unary factor g_k, so
    the factor graph is a tree and BP's marginals are exact: P(x_k) ~ u_k g_k.
    Tolerance 1e-10 absolute (sums of 1.7e6 fp64 terms per entry)."""
    import numpy as np
    k = 1291
    rng = np.random.default_rng(3)
    u = [rng.uniform(0.5, 2.0, k) for _ in range(3)]
    g = [rng.uniform(0.5, 2.0, k) for _ in range(3)]
    big = np.multiply.outer(np.multiply.outer(u[0], u[1]), u[2]).reshape(-1)
    assert big.size >= 2 ** 31
    vals = np.concatenate([big] + g)
    del big
    m = bnpp.Model.from_arrays([k, k, k], [[0, 1, 2], [0], [1], [2]], vals)
    del vals
    with _env(BNPP_BP_MODE="single"):
        with pytest.raises(bnpp.BnppError):
            bnpp.sum_product(ctx, m, 100, 1e-9)
    marg, it, _ = bnpp.sum_product(ctx, m, 100, 1e-9)
    del m
    assert 1 <= it < 100, it
    for v in range(3):
        want = u[v] * g[v]
        want = want / want.sum()
        err = float(np.max(np.abs(np.asarray(marg[v]) - want)))
        assert err <= 1e-10, (v, err)
