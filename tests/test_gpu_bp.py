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
    """Messages in global memory (BNPP_BP_NO_LDS, the path of models with more
    than 4096 message entries) give the same bits as messages in LDS."""
    import os
    m = bnpp.Model.load(model_path(model))
    lds = bnpp.sum_product(ctx, m, 10000, 1e-6)
    os.environ["BNPP_BP_NO_LDS"] = "1"
    try:
        glb = bnpp.sum_product(ctx, m, 10000, 1e-6)
    finally:
        del os.environ["BNPP_BP_NO_LDS"]
    assert lds[0] == glb[0] and lds[1] == glb[1]
