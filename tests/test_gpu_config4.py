"""BASELINE config 4 at its stated size: a Promedas-style two-layer noisy-OR BN
(50 diseases -> 80 findings, 3 parents per finding, every finding observed),
reference min-fill width 22.

Golden values come from the reference itself (tests/golden/make_golden.py
config4 -> config4_golden.json): BN::partition (model.cpp:250-301), three
single-target conditionings Z(x_t = 1), and the reference MAR of every disease
(one VE per target, model.cpp:326-334 + normalize).

Tolerances: fp64 PR bit-exact against the oracle (same min-fill order, same
chain order), 1e-12 relative against the reference (its unordered_set chain
order can change the last bit); fp32 1e-6 relative on log10 Z; marginals
1e-12 absolute (fp64) / 1e-5 (fp32) against the reference's.
"""
import json
import math
import os

import pytest

import bnpp
import refcpu
from conftest import GOLDEN, evidence_of, model_path

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c4():
    with open(os.path.join(GOLDEN, "config4_golden.json")) as f:
        g = json.load(f)
    return g, bnpp.Model.load(model_path(g["model"])), evidence_of(g["evidence"])


def test_config4_width_is_the_stated_treewidth(c4):
    g, m, ev = c4
    assert g["ref_width"] == 22
    _, w = bnpp.ordering(m, None, "mf")
    assert w == g["ref_width"]


def test_config4_partition_fp64(ctx, c4):
    g, m, ev = c4
    lz, z, _ = bnpp.partition(ctx, m, ev, "mf", bnpp.F64)
    rz, _ = refcpu.Model.load(model_path(g["model"])).partition(ev, "mf")
    assert z == rz                                                     # oracle: bit-exact
    assert abs(z - g["pr"]["Z"]) <= 1e-12 * g["pr"]["Z"]               # reference
    assert abs(lz - g["pr"]["log10Z"]) <= 1e-12 * abs(g["pr"]["log10Z"])


def test_config4_partition_fp32(ctx, c4):
    g, m, ev = c4
    lz, _, _ = bnpp.partition(ctx, m, ev, "mf", bnpp.F32)
    assert abs(lz - g["pr"]["log10Z"]) <= 1e-6 * abs(g["pr"]["log10Z"])


def test_config4_conditioned_partitions(ctx, c4):
    g, m, ev = c4
    for c in g["conditioned"]:
        e = dict(ev)
        e[c["target"]] = c["value"]
        lz, z, _ = bnpp.partition(ctx, m, e, "mf", bnpp.F64)
        assert abs(z - c["Z"]) <= 1e-12 * c["Z"], c
        lz32, _, _ = bnpp.partition(ctx, m, e, "mf", bnpp.F32)
        assert abs(lz32 - c["log10Z"]) <= 1e-6 * abs(c["log10Z"]), c


def _check_marginals(marg, g, ev, tol):
    assert len(g["marginals"]) == 50
    for t, ref in g["marginals"].items():
        t = int(t)
        assert ref["scope"] == [t]
        for a, b in zip(marg[t], ref["values"]):
            assert abs(a - b) <= tol, (t, marg[t], ref["values"])
    for v, x in ev.items():                                            # observed findings: one-hot
        assert marg[v] == [1.0 if s == x else 0.0 for s in range(2)]


@pytest.mark.parametrize("dtype,tol", [(bnpp.F64, 1e-12), (bnpp.F32, 1e-5)])
def test_config4_marginals_per_target(ctx, c4, dtype, tol):
    """BN::marginals as the reference runs it: one VE per target."""
    g, m, ev = c4
    marg, _ = bnpp.marginals(ctx, m, ev, "mf", dtype)
    _check_marginals(marg, g, ev, tol)


@pytest.mark.parametrize("dtype,tol", [(bnpp.F64, 1e-12), (bnpp.F32, 1e-5)])
def test_config4_marginals_bucket_tree(ctx, c4, dtype, tol):
    """All marginals from one two-pass bucket tree, against the reference's
    per-target MAR and against Z(x_t = 1) / Z of the golden conditionings."""
    g, m, ev = c4
    marg, _ = bnpp.marginals_tree(ctx, m, ev, "mf", dtype)
    _check_marginals(marg, g, ev, tol)
    for c in g["conditioned"]:
        p = 10 ** (c["log10Z"] - g["pr"]["log10Z"])
        assert abs(marg[c["target"]][c["value"]] - p) <= tol, c
        assert math.isclose(sum(marg[c["target"]]), 1.0, abs_tol=1e-12)
