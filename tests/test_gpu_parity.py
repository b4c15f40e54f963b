"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference's golden vectors.

Tolerances (north star: index arithmetic bit-exact, PR/MAR within 1e-6 rel):
  * fp64: bit-exact against the oracle for single ops, buckets and whole VE runs
    (same elimination order, same chain order, -ffp-contract=off kernels, exact
    power-of-two rescaling); against the reference's own golden values 1e-12
    relative on Z (the reference may multiply >=3-factor chains in another order).
  * fp32: 1e-6 relative on single-op values, 1e-6 relative on log10 Z,
    1e-5 absolute on marginals.
"""
import math
import random

import pytest
import torch

import bnpp
import refcpu
from conftest import evidence_of, model_path

pytestmark = pytest.mark.gpu

DEV = "cuda"
TD = {bnpp.F64: torch.float64, bnpp.F32: torch.float32}


_STREAM = None


def _stream():
    """A dedicated non-null torch stream shared by the tests' torch ops and the
    engine's launches (torch's default stream handle is 0, which the ABI reads
    as 'the context stream')."""
    global _STREAM
    if _STREAM is None:
        _STREAM = torch.cuda.Stream()
    torch.cuda.set_stream(_STREAM)
    return _STREAM.cuda_stream


def _dev(vals, dtype):
    return torch.tensor(vals, dtype=TD[dtype], device=DEV)


def _cards_list(cards: dict):
    n = max(cards) + 1
    return [cards.get(v, 1) for v in range(n)]


def run_bucket(ctx, dtype, cards, inputs, elim, out_vars=None, with_sum=False):
    """inputs: [(scope, values)] -> (out_scope, values list[, partition sum])"""
    scopes = [s for s, _ in inputs]
    if out_vars is None:
        out_vars = bnpp.out_scope(scopes, elim)
    size = 1
    for v in out_vars:
        size *= cards[v]
    tabs = [_dev(vals, dtype) for _, vals in inputs]
    out = torch.full((size,), float("nan"), dtype=TD[dtype], device=DEV)
    psum = torch.full((1,), float("nan"), dtype=torch.float64, device=DEV)
    bnpp.bucket_eliminate(ctx, dtype, _cards_list(cards), [t.data_ptr() for t in tabs], scopes, elim,
                          out.data_ptr(), out_vars, stream=_stream(), out_sum=psum.data_ptr() if with_sum else None)
    torch.cuda.synchronize()
    if with_sum:
        return out_vars, out.cpu().tolist(), psum.item()
    return out_vars, out.cpu().tolist()


def _check_sum(dtype, got, want, case):
    """Factor::_partition: fp64 bit-exact (same terms, same order); fp32 terms
    summed in fp64: 1e-6 relative"""
    if dtype == bnpp.F64:
        assert got == want, (case, got, want)
    else:
        assert abs(got - want) <= 1e-6 * abs(want) + 1e-30, (case, got, want)


# ------------------------------------------------------------ single ops
@pytest.mark.parametrize("dtype", [bnpp.F64, bnpp.F32])
def test_kat_single_ops(ctx, golden_kat, dtype):
    cards = {int(k): v for k, v in golden_kat["cards"].items()}
    facs = golden_kat["factors"]
    outs = golden_kat["outputs"]
    products = {}
    checked = 0
    for case in golden_kat["cases"]:
        ref = outs[case["out"]]
        op = case["op"]
        psum = None
        if op == "product":
            a, b = facs[case["a"]], facs[case["b"]]
            scope, vals, psum = run_bucket(ctx, dtype, cards, [(a["scope"], a["values"]), (b["scope"], b["values"])],
                                           -1, with_sum=True)
            products[case["out"]] = (scope, ref["values"])     # feed sum_out the reference's exact table
        elif op == "sum_out":
            s, v = products[case["a"]]
            scope, vals, psum = run_bucket(ctx, dtype, cards, [(s, v)], case["var"], with_sum=True)
        elif op == "bucket":
            ins = [(facs[x]["scope"], facs[x]["values"]) for x in case["inputs"]]
            scope, vals, psum = run_bucket(ctx, dtype, cards, ins, case["var"], with_sum=True)
        elif op == "cond":
            a = facs[case["a"]]
            ev = {int(k): v for k, v in case["evidence"].items()}
            scope = [v for v in a["scope"] if v not in ev]
            size = 1
            for v in scope:
                size *= cards[v]
            t = _dev(a["values"], dtype)
            out = torch.full((size,), float("nan"), dtype=TD[dtype], device=DEV)
            ps = torch.full((1,), float("nan"), dtype=torch.float64, device=DEV)
            bnpp.condition(ctx, dtype, _cards_list(cards), t.data_ptr(), a["scope"], ev, out.data_ptr(),
                           stream=_stream(), out_sum=ps.data_ptr())
            torch.cuda.synchronize()
            vals, psum = out.cpu().tolist(), ps.item()
        elif op == "divide":              # Factor::divide (factor.cpp:149-180), bnpp_divide
            a, b = facs[case["a"]], facs[case["b"]]
            scope = ref["scope"]
            size = 1
            for v in scope:
                size *= cards[v]
            ta, tb = _dev(a["values"], dtype), _dev(b["values"], dtype)
            out = torch.full((size,), float("nan"), dtype=TD[dtype], device=DEV)
            ps = torch.full((1,), float("nan"), dtype=torch.float64, device=DEV)
            bnpp.divide(ctx, dtype, _cards_list(cards), ta.data_ptr(), a["scope"], tb.data_ptr(), b["scope"],
                        out.data_ptr(), scope, stream=_stream(), out_sum=ps.data_ptr())
            torch.cuda.synchronize()
            vals, psum = out.cpu().tolist(), ps.item()
        else:
            continue                      # normalize: host bookkeeping (width <= 1 in MAR)
        assert scope == ref["scope"], case
        if dtype == bnpp.F64:
            assert vals == ref["values"], case
        else:
            for x, y in zip(vals, ref["values"]):
                assert abs(x - y) <= 1e-6 * abs(y) + 1e-30, (case, x, y)
        # Factor::partition() of the op (factor.cpp:139, 172, 208, 236), from the ABI's out_sum
        _check_sum(dtype, psum, ref["partition"], case)
        checked += 1
    assert checked >= 260


def _rand_bucket(rng, n_vars=12):
    cards = {v: rng.randint(2, 5) for v in range(n_vars)}
    n_in = rng.randint(1, 8)
    ins = []
    for _ in range(n_in):
        w = rng.randint(0, 4)
        scope = rng.sample(range(n_vars), w)
        size = 1
        for v in scope:
            size *= cards[v]
        ins.append((scope, [rng.uniform(0.1, 2.0) for _ in range(size)]))
    union = []
    for s, _ in ins:
        union += [v for v in s if v not in union]
    elim = rng.choice(union) if union and rng.random() < 0.8 else -1
    return cards, ins, elim


def test_random_buckets_bit_exact_vs_oracle(ctx):
    rng = random.Random(2024)
    for it in range(150):
        cards, ins, elim = _rand_bucket(rng)
        scope, vals, psum = run_bucket(ctx, bnpp.F64, cards, ins, elim, with_sum=True)
        fs = [refcpu.Factor.new(s, cards, v) for s, v in ins]
        if elim >= 0:
            ref = refcpu.bucket(fs, elim, cards[elim])
        else:
            ref = fs[0]
            for f in fs[1:]:
                ref = ref.product(f)
        assert scope == ref.scope, it
        assert vals == ref.values, it
        assert psum == ref.partition, (it, psum, ref.partition)


@pytest.mark.parametrize("k,n_other", [(2, 12), (4, 6), (2, 9)])
def test_interleaved_stream_buckets(ctx, k, n_other):
    """Stream form with the summed variable as the big input's FASTEST dim and
    the output's dim 0 right above it (the backward messages of a column-sweep
    bucket tree): bit-exact against the oracle in fp64, 1e-6 in fp32."""
    rng = random.Random(k * 100 + n_other)
    y = 0
    others = list(range(1, n_other + 2))
    cards = {y: k}
    for v in others:
        cards[v] = rng.choice([2, 3, 4])
    cards[others[-1]] = 4                     # output dim 0: a multiple of the tile width
    big_scope = others + [y]
    size = 1
    for v in big_scope:
        size *= cards[v]
    big = (big_scope, [rng.uniform(0.5, 2.0) for _ in range(size)])
    pair = ([others[-1], y], [rng.uniform(0.5, 2.0) for _ in range(4 * k)])
    unary = ([y], [rng.uniform(0.5, 2.0) for _ in range(k)])
    for ins in ([big, pair], [pair, big, unary], [unary, big]):
        fs = [refcpu.Factor.new(sc, cards, v) for sc, v in ins]
        ref = refcpu.bucket(fs, y, cards[y])
        scope, vals = run_bucket(ctx, bnpp.F64, cards, ins, y)
        assert scope == ref.scope
        assert vals == ref.values
        scope, vals = run_bucket(ctx, bnpp.F32, cards, ins, y)
        assert max(abs(a - b) / abs(b) for a, b in zip(vals, ref.values)) < 1e-6


@pytest.mark.parametrize("k,kq,n_other", [(2, 2, 12), (2, 4, 8), (4, 2, 6), (4, 4, 5)])
def test_interleaved_broadcast_rows(ctx, k, kq, n_other):
    """The tree's backward message: the parent variable xq is absent from the
    big input and is the output's SLOWEST dim; the tile spans xq so one load of
    the big values serves every row (output rows at xq's stride).  Compared
    with the oracle's table (reference order) transposed to the planned layout."""
    rng = random.Random(k * 1000 + kq * 100 + n_other)
    xq, y = 0, 1
    others = list(range(2, n_other + 2))
    cards = {xq: kq, y: k}
    for v in others:
        cards[v] = rng.choice([2, 4])
    cards[others[-1]] = 4
    size = k
    for v in others:
        size *= cards[v]
    big = (others + [y], [rng.uniform(0.5, 2.0) for _ in range(size)])
    pair = ([xq, y], [rng.uniform(0.5, 2.0) for _ in range(kq * k)])
    side = ([xq, others[-1]], [rng.uniform(0.5, 2.0) for _ in range(kq * 4)])
    unary = ([xq], [rng.uniform(0.5, 2.0) for _ in range(kq)])
    ins = [big, pair, side, unary]
    fs = [refcpu.Factor.new(sc, cards, v) for sc, v in ins]
    ref = refcpu.bucket(fs, y, cards[y])
    planned = [xq] + others
    t = torch.tensor(ref.values, dtype=torch.float64).reshape([cards[v] for v in ref.scope])
    want = t.permute([ref.scope.index(v) for v in planned]).reshape(-1).tolist()
    scope, vals = run_bucket(ctx, bnpp.F64, cards, ins, y, out_vars=planned)
    assert scope == planned
    assert vals == want
    scope, vals = run_bucket(ctx, bnpp.F32, cards, ins, y, out_vars=planned)
    assert max(abs(a - b) / abs(b) for a, b in zip(vals, want)) < 1e-6


@pytest.mark.parametrize("k,c0,scards", [(4, 4, [4] * 6), (2, 2, [2] * 13), (2, 4, [2] * 12), (3, 1, [3] * 8),
                                         (1, 2, [2] * 13), (2, 2, [3] * 8), (4, 1, [2] * 12), (3, 4, [3, 2] * 4)])
def test_slab_form_buckets(ctx, k, c0, scards):
    """Slab form (slab.cuh, flat grid): the big input holds the summed variable
    x as its slowest dim (k slabs contiguous along the output's slow index S),
    small inputs depend on (x, y) only, the output is (S..., y).  Every chain
    position of the big input; odd S cards force the one-entry-per-lane tile.
    fp64 bit-exact against the oracle, fp32 1e-6 relative."""
    rng = random.Random(k * 1000 + c0 * 100 + len(scards))
    x, y = 0, 1
    S = list(range(2, 2 + len(scards)))
    cards = {x: k, y: c0}
    for v, c in zip(S, scards):
        cards[v] = c
    size = k
    for c in scards:
        size *= c
    big = ([x] + S, [rng.uniform(0.5, 2.0) for _ in range(size)])
    ys = [y] if c0 > 1 else []
    pair = ([x] + ys, [rng.uniform(0.5, 2.0) for _ in range(k * c0)])
    unary = ([x], [rng.uniform(0.5, 2.0) for _ in range(k)])
    side = (ys, [rng.uniform(0.5, 2.0) for _ in range(c0)])
    elim = x if k > 1 else -1
    for ins in ([big, pair], [pair, big], [unary, big, pair], [unary, pair, big, side], [big, side, unary]):
        fs = [refcpu.Factor.new(sc, cards, v) for sc, v in ins]
        if elim >= 0:
            ref = refcpu.bucket(fs, elim, k)
        else:
            ref = fs[0]
            for f in fs[1:]:
                ref = ref.product(f)
        planned = S + ys + ([x] if elim < 0 else [])
        t = torch.tensor(ref.values, dtype=torch.float64).reshape([cards[v] for v in ref.scope])
        want = t.permute([ref.scope.index(v) for v in planned]).reshape(-1).tolist()
        scope, vals = run_bucket(ctx, bnpp.F64, cards, ins, elim, out_vars=planned)
        assert vals == want, [s for s, _ in ins]
        scope, vals = run_bucket(ctx, bnpp.F32, cards, ins, elim, out_vars=planned)
        assert max(abs(a - b) / abs(b) for a, b in zip(vals, want)) < 1e-6


@pytest.mark.parametrize("n_small,big_at", [(4, 0), (4, 3), (5, 2), (7, 7), (6, 1)])
def test_stream_buckets_five_to_eight_inputs(ctx, n_small, big_at):
    """Stream form with 5-8 inputs (kStream8In: one big input streamed, 4-7
    small ones from LDS) -- the conditioned 32x32 PR's 5-input bucket over an
    8-GiB message.  Small inputs over the output's fastest dims, the summed
    variable and a slow dim; the big one at every chain position.  fp64
    bit-exact against the oracle (and its partition sum), fp32 1e-6."""
    rng = random.Random(n_small * 10 + big_at)
    x, a, b, z = 0, 1, 2, 3                       # summed var; fastest output dims a, b; slow dim z
    mid = list(range(4, 15))                      # the big input's middle dims (>= 2^13 entries)
    cards = {x: 2, a: 2, b: 2, z: 2}
    for v in mid:
        cards[v] = rng.choice([2, 3])
    bs = [z] + mid + [x]
    size = 1
    for v in bs:
        size *= cards[v]
    big = (bs, [rng.uniform(0.5, 2.0) for _ in range(size)])
    pool = [[x, a], [x, b], [z, x], [a], [b, x], [x], [a, b], [z, a]]
    smalls = []
    for i in range(n_small):
        sc = pool[i % len(pool)]
        n = 1
        for v in sc:
            n *= cards[v]
        smalls.append((sc, [rng.uniform(0.5, 2.0) for _ in range(n)]))
    ins = smalls[:big_at] + [big] + smalls[big_at:]
    fs = [refcpu.Factor.new(sc, cards, v) for sc, v in ins]
    ref = refcpu.bucket(fs, x, cards[x])
    planned = [z] + mid + [b, a]
    t = torch.tensor(ref.values, dtype=torch.float64).reshape([cards[v] for v in ref.scope])
    want = t.permute([ref.scope.index(v) for v in planned]).reshape(-1).tolist()
    scope, vals = run_bucket(ctx, bnpp.F64, cards, ins, x, out_vars=planned)
    assert vals == want
    scope, vals = run_bucket(ctx, bnpp.F32, cards, ins, x, out_vars=planned)
    assert max(abs(p - q) / abs(q) for p, q in zip(vals, want)) < 1e-6
    # the whole-table partition sum in the reference's (entry, value) order
    scope, vals, psum2 = run_bucket(ctx, bnpp.F64, cards, ins, x, with_sum=True)
    assert vals == ref.values and psum2 == ref.partition


@pytest.mark.parametrize("n_small,big_at", [(2, 0), (2, 1), (3, 2), (4, 0), (4, 4), (5, 3), (7, 1)])
def test_slab_rows_over_two_dims(ctx, n_small, big_at):
    """Slab form whose tile row spans the output's two fastest (binary) dims,
    which the big input does not vary along (slab_y2), with 2-8 inputs
    (kSlab8In from 5): the big input holds x as slabs contiguous along the
    output's slow index, the small inputs depend on (x, a, b).  fp64
    bit-exact against the oracle, fp32 1e-6."""
    rng = random.Random(700 + n_small * 10 + big_at)
    x, a, b = 0, 1, 2
    mid = list(range(3, 15))
    cards = {x: 2, a: 2, b: 2}
    for v in mid:
        cards[v] = rng.choice([2, 3])
    cards[mid[-1]] = 4                            # whole tiles: the slab dim is a multiple of 4
    size = 2
    for v in mid:
        size *= cards[v]
    big = ([x] + mid, [rng.uniform(0.5, 2.0) for _ in range(size)])
    pool = [[x, a], [b, x], [a, b], [x], [x, a, b], [a], [b, a, x]]
    smalls = []
    for i in range(n_small):
        sc = pool[i % len(pool)]
        n = 1
        for v in sc:
            n *= cards[v]
        smalls.append((sc, [rng.uniform(0.5, 2.0) for _ in range(n)]))
    ins = smalls[:big_at] + [big] + smalls[big_at:]
    fs = [refcpu.Factor.new(sc, cards, v) for sc, v in ins]
    ref = refcpu.bucket(fs, x, cards[x])
    planned = mid + [b, a]
    t = torch.tensor(ref.values, dtype=torch.float64).reshape([cards[v] for v in ref.scope])
    want = t.permute([ref.scope.index(v) for v in planned]).reshape(-1).tolist()
    scope, vals = run_bucket(ctx, bnpp.F64, cards, ins, x, out_vars=planned)
    assert vals == want
    scope, vals = run_bucket(ctx, bnpp.F32, cards, ins, x, out_vars=planned)
    assert max(abs(p - q) / abs(q) for p, q in zip(vals, want)) < 1e-6


def test_slab_level_kernels_in_ve(ctx, monkeypatch, capfd):
    """Whole VE runs with fused sweep runs off: a 12x12 min-fill plan and a
    14x14 column sweep hold slab-form buckets (bcls 8 in the plan dump), run by
    the slab level kernel (flat grid, rescaling, max tracking).  fp64 log10 Z
    identical with the slab form off, and the oracle's within 1e-13."""
    from bnpp import synth
    monkeypatch.setenv("BNPP_NO_CHAIN", "1")
    for n, order in ((12, None), (14, [r * 14 + c for c in range(14) for r in range(14)])):
        d = synth.ising_grid(n, n, seed=3)
        m = bnpp.Model.from_dict(d)
        monkeypatch.setenv("BNPP_DUMP_PLAN", "1")
        capfd.readouterr()
        lz_slab = bnpp.partition(ctx, m, {}, "mf", bnpp.F64, order=order)[0]
        assert "bcls=8" in capfd.readouterr().err
        monkeypatch.delenv("BNPP_DUMP_PLAN")
        monkeypatch.setenv("BNPP_NO_SLAB", "1")
        lz_gen = bnpp.partition(ctx, m, {}, "mf", bnpp.F64, order=order)[0]
        monkeypatch.delenv("BNPP_NO_SLAB")
        assert lz_slab == lz_gen
        if order is None:
            rz = refcpu.Model.from_dict(d).partition({}, "mf")[0]
            assert abs(math.log10(rz) - lz_slab) < 1e-13
        f32 = bnpp.partition(ctx, m, {}, "mf", bnpp.F32, order=order)[0]
        assert abs(f32 - lz_slab) < 1e-6 * abs(lz_slab)


def test_permuted_output_layout(ctx):
    """Any permutation of the output scope is accepted and gives the same table, transposed."""
    rng = random.Random(5)
    for it in range(30):
        cards, ins, elim = _rand_bucket(rng, 8)
        scope, vals = run_bucket(ctx, bnpp.F64, cards, ins, elim)
        if len(scope) < 2:
            continue
        perm = scope[:]
        rng.shuffle(perm)
        pscope, pvals = run_bucket(ctx, bnpp.F64, cards, ins, elim, out_vars=perm)
        t = torch.tensor(vals, dtype=torch.float64).reshape([cards[v] for v in scope])
        t = t.permute([scope.index(v) for v in perm]).reshape(-1)
        assert pvals == t.tolist(), it


def test_sum_out_absent_variable_is_copy(ctx):
    cards = {0: 3, 1: 2, 2: 4}
    vals = [float(i + 1) for i in range(6)]
    scope, out = run_bucket(ctx, bnpp.F64, cards, [([0, 1], vals)], 2)
    assert scope == [0, 1] and out == vals


def test_width_zero_and_unit_factors(ctx):
    cards = {0: 2, 1: 3}
    scope, out = run_bucket(ctx, bnpp.F64, cards, [([], [2.5]), ([], [4.0])], -1)
    assert scope == [] and out == [10.0]
    scope, out = run_bucket(ctx, bnpp.F64, cards, [([], [2.0]), ([0], [1.0, 3.0])], 0)
    assert scope == [] and out == [8.0]


def test_invalid_shapes_rejected(ctx):
    a = _dev([1.0, 2.0], bnpp.F64)
    out = _dev([0.0, 0.0], bnpp.F64)
    with pytest.raises(bnpp.BnppError) as e:       # output scope is not union minus elim
        bnpp.bucket_eliminate(ctx, bnpp.F64, [2, 2], [a.data_ptr()], [[0]], -1, out.data_ptr(), [1])
    assert e.value.status == bnpp.ERR_INVALID
    with pytest.raises(bnpp.BnppError):            # more than 8 inputs
        bnpp.bucket_eliminate(ctx, bnpp.F64, [2], [a.data_ptr()] * 9, [[0]] * 9, -1, out.data_ptr(), [0])
    # variable ids outside cards[0, n_cards) are rejected before cards is read
    for scope, elim, ov in (([2], -1, [2]), ([0], 5, [0]), ([-1], -1, [-1]), ([0], -1, [3])):
        with pytest.raises(bnpp.BnppError) as e:
            bnpp.bucket_eliminate(ctx, bnpp.F64, [2, 2], [a.data_ptr()], [scope], elim, out.data_ptr(), ov)
        assert e.value.status == bnpp.ERR_INVALID, (scope, elim, ov)
    with pytest.raises(bnpp.BnppError) as e:
        bnpp.divide(ctx, bnpp.F64, [2], a.data_ptr(), [0], a.data_ptr(), [1], out.data_ptr(), [0, 1])
    assert e.value.status == bnpp.ERR_INVALID
    with pytest.raises(bnpp.BnppError) as e:
        bnpp.condition(ctx, bnpp.F64, [2], a.data_ptr(), [4], {}, out.data_ptr())
    assert e.value.status == bnpp.ERR_INVALID


# ----------------------------------------------------------- whole VE runs
FAST_PR = [c for c in ["grid3x3.uai", "network.uai", "asia.uai", "potts6x6.uai", "potts4x5k3.uai", "ising4x4.uai",
                       "ising5x5.uai", "ising6x6.uai", "ising8x8.uai", "ising10x10.uai", "ising12x12.uai",
                       "cancer.uai", "earthquake.uai", "child.uai", "alarm.uai", "insurance.uai", "hailfinder.uai",
                       "noisyor_30_40.uai", "pathfinder.uai", "Water.uai", "hepar2.uai", "win95pts.uai",
                       "andes.uai"]]


def _pr_cases(golden_ve, models=None):
    return [c for c in golden_ve["pr"] if models is None or c["model"] in models]


def test_partition_fp64_bit_exact(ctx, golden_ve):
    n = 0
    for case in _pr_cases(golden_ve, FAST_PR):
        m = bnpp.Model.load(model_path(case["model"]))
        ev = evidence_of(case["evidence"])
        lz, z, _ = bnpp.partition(ctx, m, ev, case["heuristic"], bnpp.F64)
        rz, _ = refcpu.Model.load(model_path(case["model"])).partition(ev, case["heuristic"])
        assert z == rz, (case, z, rz)                                     # oracle: bit-exact
        assert abs(z - case["Z"]) <= 1e-12 * abs(case["Z"]), (case, z)     # reference: chain-order rounding
        assert abs(lz - math.log10(rz)) <= 1e-12 * max(1.0, abs(lz))
        n += 1
    assert n >= 20


def test_partition_strip_12x32(ctx, golden_ve):
    """BASELINE config 3 restated: the reference-runnable 32x12 strip."""
    case = _pr_cases(golden_ve, {"ising12x32.uai"})[0]
    m = bnpp.Model.load(model_path(case["model"]))
    lz, z, _ = bnpp.partition(ctx, m, {}, "mf", bnpp.F64)
    assert abs(z - case["Z"]) <= 1e-12 * abs(case["Z"])
    lz32, _, _ = bnpp.partition(ctx, m, {}, "mf", bnpp.F32)
    assert abs(lz32 - case["log10Z"]) <= 1e-6 * abs(case["log10Z"])


def test_partition_fp32_within_tolerance(ctx, golden_ve):
    for case in _pr_cases(golden_ve, FAST_PR):
        m = bnpp.Model.load(model_path(case["model"]))
        lz, _, _ = bnpp.partition(ctx, m, evidence_of(case["evidence"]), case["heuristic"], bnpp.F32)
        assert abs(lz - case["log10Z"]) <= 1e-6 * max(1.0, abs(case["log10Z"])), (case, lz)


@pytest.mark.parametrize("dtype", [bnpp.F64, bnpp.F32])
def test_marginals_vs_golden(ctx, golden_ve, dtype):
    for case in golden_ve["mar"]:
        m = bnpp.Model.load(model_path(case["model"]))
        ev = evidence_of(case["evidence"])
        marg, _ = bnpp.marginals(ctx, m, ev, case["heuristic"], dtype)
        if dtype == bnpp.F64:
            rm, _ = refcpu.Model.load(model_path(case["model"])).marginals(ev, case["heuristic"])
        for t, ref in case["marginals"].items():
            t = int(t)
            if not ref["scope"]:
                assert marg[t][ev[t]] == 1.0 and sum(marg[t]) == 1.0
                continue
            if dtype == bnpp.F64:
                assert marg[t] == rm[t], (case["model"], t)                # oracle: bit-exact
                tol = 1e-13
            else:
                tol = 1e-5
            for a, b in zip(marg[t], ref["values"]):
                assert abs(a - b) <= tol, (case["model"], t, marg[t], ref["values"])


def test_reference_fixture_files(ctx):
    """models/markovnets/grid3x3.uai.PR = 14.8899, network.uai.PR = 163.204 (log10 Z)."""
    for name, ev in (("grid3x3.uai", "grid3x3-PR.uai.evid"), ("network.uai", "network.uai.evid")):
        m = bnpp.Model.load(model_path(name))
        lz, _, _ = bnpp.partition(ctx, m, bnpp.load_evidence(model_path(ev)), "mf", bnpp.F64)
        want = float(open(model_path(name + ".PR")).read().split()[-1])
        assert round(lz, 4 if abs(want) < 100 else 3) == want


def test_job_relaunch_is_idempotent(ctx):
    m = bnpp.Model.load(model_path("ising10x10.uai"))
    job = bnpp.Job(ctx, m, "pr", heuristic="mf", dtype=bnpp.F64)
    job.launch()
    a = job.results()
    for _ in range(3):
        job.launch()
    b = job.results()
    assert a == b
    job.close()


# ------------------------------------------------ size-independent properties
def test_order_independence_20x20(ctx):
    """log10 Z of a 20x20 grid (beyond the oracle's reach) agrees across
    elimination orders (different buckets, layouts and message shapes)."""
    from bnpp import synth
    m = bnpp.Model.from_dict(synth.ising_grid(20, 20, seed=3))
    vals = [bnpp.partition(ctx, m, {}, h, bnpp.F64)[0] for h in ("mf", "wmf", "md")]
    col = [c * 20 + r for c in range(20) for r in range(20)]                 # column sweep, width 20
    vals.append(bnpp.partition(ctx, m, {}, "mf", bnpp.F64, order=col)[0])
    for v in vals[1:]:
        assert abs(v - vals[0]) <= 1e-10 * abs(vals[0]), vals
    v32 = bnpp.partition(ctx, m, {}, "mf", bnpp.F32)[0]
    assert abs(v32 - vals[0]) <= 1e-6 * abs(vals[0])


def test_marginals_normalised_and_consistent_14x14(ctx):
    """MAR on a 14x14 grid: every marginal sums to 1, and the marginal of the
    last variable matches Z(x=k)/Z computed by conditioned partitions."""
    from bnpp import synth
    m = bnpp.Model.from_dict(synth.ising_grid(14, 14, seed=4))
    marg, _ = bnpp.marginals(ctx, m, {}, "mf", bnpp.F64)
    for t, p in marg.items():
        assert abs(sum(p) - 1.0) < 1e-12
    lz = bnpp.partition(ctx, m, {}, "mf", bnpp.F64)[0]
    t = 195
    for k in range(2):
        lzk = bnpp.partition(ctx, m, {t: k}, "mf", bnpp.F64)[0]
        assert abs(10 ** (lzk - lz) - marg[t][k]) < 1e-12


@pytest.mark.parametrize("k,w", [(2, 22), (4, 11)])
def test_micro_bucket_checksum(ctx, k, w):
    """Fused m(x,S)*f(x,y) -> sum_x at large size: checksum of checksums
    sum_out = sum_x (sum_S m[x,S]) * (sum_y f[x,y]), plus sampled entries."""
    g = torch.Generator(device=DEV).manual_seed(0)
    S = k ** w
    for dtype in (bnpp.F64, bnpp.F32):
        m_t = torch.rand(k * S, generator=g, device=DEV, dtype=TD[dtype]) * 1.5 + 0.5
        f_t = torch.rand(k * k, generator=g, device=DEV, dtype=TD[dtype]) * 1.5 + 0.5
        out = torch.empty(S * k, device=DEV, dtype=TD[dtype])
        cards = [k] * (w + 2)
        sm = list(range(w + 1))
        sf = [0, w + 1]
        bnpp.bucket_eliminate(ctx, dtype, cards, [m_t.data_ptr(), f_t.data_ptr()], [sm, sf], 0, out.data_ptr(),
                              list(range(1, w + 2)), stream=_stream())
        torch.cuda.synchronize()
        M = m_t.double().reshape(k, S)
        F = f_t.double().reshape(k, k)
        want = (M.sum(1) * F.sum(1)).sum().item()
        got = out.double().sum().item()
        assert abs(got - want) <= (1e-9 if dtype == bnpp.F64 else 1e-4) * want
        idx = torch.randint(0, S * k, (4096,), generator=g, device=DEV)
        s_i, y_i = idx // k, idx % k
        ref = (M[:, s_i] * F[:, y_i]).sum(0)
        assert torch.allclose(out[idx].double(), ref, rtol=1e-12 if dtype == bnpp.F64 else 1e-6)
        del m_t, out


def test_bench_bucket_full_size_exact(ctx):
    """The bench's bucket at its full size (BASELINE config 5 restated: k = 4,
    |S| = 14, fp32, 4^16 factor-entries, 4.3 GB in and out): checksum of
    checksums, and 4096 sampled entries equal -- bit for bit -- to the
    reference's arithmetic in fp32 (acc = 0; acc += m[x,s] * f[x,y] for x =
    0..k-1, each product and sum rounded, factor.cpp:131-143, 199-205)."""
    k, w = 4, 14
    S = k ** w
    g = torch.Generator(device=DEV).manual_seed(5)
    m_t = torch.rand(k * S, generator=g, device=DEV, dtype=torch.float32) * 1.5 + 0.5
    f_t = torch.rand(k * k, generator=g, device=DEV, dtype=torch.float32) * 1.5 + 0.5
    out = torch.empty(S * k, device=DEV, dtype=torch.float32)
    bnpp.bucket_eliminate(ctx, bnpp.F32, [k] * (w + 2), [m_t.data_ptr(), f_t.data_ptr()],
                          [list(range(w + 1)), [0, w + 1]], 0, out.data_ptr(), list(range(1, w + 2)),
                          stream=_stream())
    torch.cuda.synchronize()
    M, F = m_t.reshape(k, S), f_t.reshape(k, k)
    want = (M.double().sum(1) * F.double().sum(1)).sum().item()
    assert abs(out.double().sum().item() - want) <= 1e-4 * want
    idx = torch.randint(0, S * k, (4096,), generator=g, device=DEV)
    s_i, y_i = idx // k, idx % k
    acc = torch.zeros(4096, device=DEV, dtype=torch.float32)
    for x in range(k):
        acc = acc + M[x, s_i] * F[x, y_i]
    assert torch.equal(out[idx], acc)
    del m_t, out


def test_partition_corpus_matches_reference(ctx):
    """The reference's larger networks (Pigs, Link, Munin1-4, Barley, Mildew,
    Diabetes; with and without evidence): fp64 log10 Z against BN::partition's
    (tests/golden/corpus_golden.json).  Orderings may break min-fill ties
    differently (graph.cpp:50-58 iterates an unordered_set), so the products
    run in another order: 1e-9 in log10 Z."""
    import json
    import os
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "corpus_golden.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        m = bnpp.Model.load(model_path(c["model"]))
        lz, _, _ = bnpp.partition(ctx, m, evidence_of(c["evidence"]), "mf", bnpp.F64)
        assert abs(lz - c["log10Z"]) <= 1e-9, (c["model"], c["evidence"], lz, c["log10Z"])


def test_source_cache_never_serves_another_model(ctx):
    """The context keeps uploaded sources per model (capi.cpp cached_sources):
    repeated calls reuse them, and a model with the same shape but other
    values -- created after the first is freed, possibly at the same address
    -- gets its own (model uids are never reused)."""
    from bnpp import synth
    outs = []
    for seed in (1, 2, 1):
        d = synth.ising_grid(5, 6, seed=seed)
        m = bnpp.Model.from_dict(d)
        z1 = bnpp.partition(ctx, m, {}, "mf", bnpp.F64)[1]
        z2 = bnpp.partition(ctx, m, {}, "mf", bnpp.F64)[1]
        rz, _ = refcpu.Model.from_dict(d).partition({}, "mf")
        assert z1 == z2 == rz, (seed, z1, z2, rz)
        outs.append(z1)
        del m
    assert outs[0] == outs[2] and outs[0] != outs[1]


def test_variable_elimination_large_result_vs_oracle(ctx):
    """BN::variable_elimination leaving 22 of a 6x7 grid's variables: a
    4-Mi-entry result table, copied out of the arena by several workgroups
    (launch.hip copy_tables_kernel); scope in the reference's order and
    values (scaled by 2^exp2, exact) equal to the oracle's."""
    from bnpp import synth
    d = synth.ising_grid(6, 7, seed=21)
    m = bnpp.Model.from_dict(d)
    elim = list(range(0, 42, 2))[:20]
    scope, vals, e2 = bnpp.variable_elimination(ctx, m, elim, "given", bnpp.F64, cap_values=1 << 23)
    ref = refcpu.Model.from_dict(d).variable_elimination(elim, "given")
    assert scope == ref.scope
    rv = ref.values
    assert len(vals) == len(rv) == 1 << 22
    assert all(math.ldexp(a, e2) == b for a, b in zip(vals, rv))


def test_job_cache_reuses_only_identical_calls(ctx):
    """The context keeps the last one-shot job (capi.cpp oneshot_job): an
    identical call relaunches it (no planning: plan_ms 0), any difference --
    evidence, dtype, order, a BNPP_* knob -- plans afresh; results always
    equal the oracle's."""
    from bnpp import synth
    import os
    d = synth.ising_grid(6, 6, seed=4)
    m = bnpp.Model.from_dict(d)
    rm = refcpu.Model.from_dict(d)
    z0 = bnpp.partition(ctx, m, {}, "mf", bnpp.F64)[1]
    z1 = bnpp.partition(ctx, m, {}, "mf", bnpp.F64)[1]
    assert bnpp.last_timing()["plan_ms"] == 0.0
    assert z0 == z1 == rm.partition({}, "mf")[0]
    ze = bnpp.partition(ctx, m, {3: 1}, "mf", bnpp.F64)[1]
    assert bnpp.last_timing()["plan_ms"] > 0.0
    assert ze == rm.partition({3: 1}, "mf")[0]
    os.environ["BNPP_NO_CHAIN"] = "1"
    try:
        zk = bnpp.partition(ctx, m, {3: 1}, "mf", bnpp.F64)[1]
        assert bnpp.last_timing()["plan_ms"] > 0.0
    finally:
        del os.environ["BNPP_NO_CHAIN"]
    assert zk == ze
    mg = bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F64)[0]
    mg2 = bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F64)[0]
    assert bnpp.last_timing()["plan_ms"] == 0.0 and mg == mg2
    want, _ = rm.marginals({}, "mf")
    for t in range(m.n_vars):
        assert all(abs(a - b) <= 1e-12 for a, b in zip(mg[t], want[t]))


def test_job_cache_tolerates_budget_jitter(ctx):
    """The plan depends on the memory budget (free device memory): an identical
    call after free memory moved by < 2 % (another allocation on the device)
    still relaunches the cached job; a move of ~10 % plans afresh (capi.cpp
    same_budget).  Results equal either way."""
    import os
    import torch
    from bnpp import synth
    if os.environ.get("BNPP_MEM_BUDGET_GB"):
        pytest.skip("explicit budget")
    m = bnpp.Model.from_dict(synth.ising_grid(6, 6, seed=7))
    z0 = bnpp.partition(ctx, m, {1: 0}, "mf", bnpp.F64)[1]
    assert bnpp.last_timing()["plan_ms"] > 0.0
    free = torch.cuda.mem_get_info(0)[0]
    small = torch.empty(int(free * 0.005), dtype=torch.uint8, device="cuda:0")
    z1 = bnpp.partition(ctx, m, {1: 0}, "mf", bnpp.F64)[1]
    assert bnpp.last_timing()["plan_ms"] == 0.0 and z1 == z0
    big = torch.empty(int(free * 0.1), dtype=torch.uint8, device="cuda:0")
    z2 = bnpp.partition(ctx, m, {1: 0}, "mf", bnpp.F64)[1]
    assert bnpp.last_timing()["plan_ms"] > 0.0 and z2 == z0
    del small, big
    torch.cuda.empty_cache()


def test_job_cache_never_serves_invalid_evidence(ctx):
    """A valid one-shot call leaves its job cached; a following call with
    out-of-range evidence (a variable past the model, a negative or too large
    value) must fail with BNPP_ERR_INVALID, not relaunch the cached job
    (capi.cpp call_key validates the evidence like evidence_array)."""
    from bnpp import synth
    d = synth.ising_grid(4, 5, seed=3)
    m = bnpp.Model.from_dict(d)
    for kind in ("pr", "mar", "tree"):
        call = {"pr": lambda ev: bnpp.partition(ctx, m, ev, "mf", bnpp.F64),
                "mar": lambda ev: bnpp.marginals(ctx, m, ev, "mf", bnpp.F64),
                "tree": lambda ev: bnpp.marginals_tree(ctx, m, ev, "mf", bnpp.F64)}[kind]
        call({})
        call({})
        assert bnpp.last_timing()["plan_ms"] == 0.0        # cached
        for bad in ({999: 0}, {2: -1}, {2: 2}):
            with pytest.raises(bnpp.BnppError):
                call(bad)
        call({})


def test_model_free_releases_cached_job_and_sources(ctx):
    """bnpp_model_free drops the contexts' cached sources and one-shot job of
    the freed model (capi.cpp): later calls on other models are unaffected and
    still equal the oracle."""
    from bnpp import synth
    import gc
    d = synth.ising_grid(5, 5, seed=9)
    m = bnpp.Model.from_dict(d)
    z = bnpp.partition(ctx, m, {}, "mf", bnpp.F64)[1]
    bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F64)
    del m
    gc.collect()
    m2 = bnpp.Model.from_dict(d)
    z2 = bnpp.partition(ctx, m2, {}, "mf", bnpp.F64)[1]
    assert bnpp.last_timing()["plan_ms"] > 0.0             # a new model: planned afresh
    assert z == z2 == refcpu.Model.from_dict(d).partition({}, "mf")[0]


def test_generic_offsets_32_and_64_bit_identical(ctx, monkeypatch):
    """The generic gather kernels take 32-bit table offsets when every input
    of a launch is under 4 GiB (kGenericO32) and 64-bit ones otherwise;
    BNPP_NO_O32=1 forces the 64-bit kernels everywhere.  Same bits either way:
    PRs whose largest buckets are whole-dim odd tiles (Munin1: card-7 rows),
    a corpus network with evidence, per-target marginals, and random single
    buckets against the oracle."""
    cases = [("Munin1.uai", None), ("Pigs.uai", "Pigs.uai.evid"), ("alarm.uai", "alarm.uai.evid")]
    runs = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("BNPP_NO_O32", flag)
        out = []
        for name, evn in cases:
            m = bnpp.Model.load(model_path(name))
            ev = evidence_of(evn) if evn else {}
            for dt in (bnpp.F64, bnpp.F32):
                out.append(bnpp.partition(ctx, m, ev, "mf", dt)[:2])
        m = bnpp.Model.load(model_path("alarm.uai"))
        out.append(bnpp.marginals(ctx, m, {}, "mf", bnpp.F64)[0])
        rng = random.Random(77)
        for it in range(40):
            cards, ins, elim = _rand_bucket(rng)
            scope, vals, psum = run_bucket(ctx, bnpp.F64, cards, ins, elim, with_sum=True)
            fs = [refcpu.Factor.new(s, cards, v) for s, v in ins]
            ref = refcpu.bucket(fs, elim, cards[elim]) if elim >= 0 else fs[0]
            if elim < 0:
                for f in fs[1:]:
                    ref = ref.product(f)
            assert vals == ref.values, (flag, it)
            out.append((scope, vals, psum))
        runs[flag] = out
    assert runs["0"] == runs["1"]
