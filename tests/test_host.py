"""CPU tests of the product library's host side: the C ABI exports, loud
failure without a GPU, scope rules, UAI/evidence loading, ordering, planning."""
import os
import re

import pytest

import bnpp
import refcpu
from bnpp import synth
from conftest import REPO, evidence_of, model_path


def _header_functions():
    txt = open(os.path.join(REPO, "include", "bnpp.h")).read()
    return sorted(set(re.findall(r"^(?:int|const char \*|const char\*)\s*(bnpp_\w+)\(", txt, re.M)))


def test_library_exports_every_header_symbol():
    names = _header_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(bnpp._lib, n), n
    # and the Python binding declares them all
    assert set(names) <= set(bnpp.EXPORTED)


def test_no_cpu_fallback_without_gpu():
    if bnpp.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(bnpp.BnppError) as e:
        bnpp.Context(0)
    assert e.value.status == bnpp.ERR_NO_DEVICE


def test_out_scope_matches_reference_rules(golden_kat):
    facs = golden_kat["factors"]
    outs = golden_kat["outputs"]
    scopes = {}
    for case in golden_kat["cases"]:
        ref = outs[case["out"]]["scope"]
        if case["op"] == "product":
            s = bnpp.out_scope([facs[case["a"]]["scope"], facs[case["b"]]["scope"]])
            scopes[case["out"]] = s
            assert s == ref
        elif case["op"] == "sum_out":
            assert bnpp.out_scope([scopes[case["a"]]], case["var"]) == ref
        elif case["op"] == "bucket":
            assert bnpp.out_scope([facs[x]["scope"] for x in case["inputs"]], case["var"]) == ref


@pytest.mark.parametrize("name", ["grid3x3.uai", "network.uai", "asia.uai", "alarm.uai", "pathfinder.uai",
                                  "ising12x32.uai", "potts6x6.uai", "noisyor_30_40.uai"])
def test_uai_loader(name):
    m = bnpp.Model.load(model_path(name))
    py = synth.read_uai(model_path(name))
    assert m.n_vars == len(py["cards"])
    assert m.n_factors == len(py["scopes"])
    assert m.cards == py["cards"]
    assert m.is_bayes == (py["type"] == "BAYES")


def test_uai_loader_errors(tmp_path):
    with pytest.raises(bnpp.BnppError) as e:
        bnpp.Model.load(str(tmp_path / "missing.uai"))
    assert e.value.status == bnpp.ERR_IO
    bad = tmp_path / "bad.uai"
    bad.write_text("MARKOV\n2\n2 2\n1\n2 0 1\n3\n1 2 3\n")      # 3 values for a 4-entry table
    with pytest.raises(bnpp.BnppError):
        bnpp.Model.load(str(bad))
    hdr = tmp_path / "hdr.uai"
    hdr.write_text("# comment line\nMARKOV # trailing\n1\n2\n1\n1 0\n2\n0.5 # c\n 1.5\n")
    m = bnpp.Model.load(str(hdr))
    assert m.n_vars == 1 and m.cards == [2]


def test_evidence_loader(tmp_path):
    for name in ("grid3x3-PR.uai.evid", "grid3x3-MAR.uai.evid", "asia.uai.evid", "network.uai.evid"):
        assert bnpp.load_evidence(model_path(name)) == synth.read_evidence(model_path(name))
    p = tmp_path / "two.evid"
    p.write_text("2\n1 0 1\n")          # sample count != 1: nothing is read (io.cpp:164)
    assert bnpp.load_evidence(str(p)) == {}


@pytest.mark.parametrize("name", ["ising8x8.uai", "ising10x10.uai", "ising12x32.uai", "network.uai", "alarm.uai",
                                  "potts6x6.uai", "hailfinder.uai", "noisyor_30_40.uai"])
@pytest.mark.parametrize("h", ["mf", "wmf", "md"])
def test_ordering_identical_to_oracle(name, h):
    """Same selection rules and tie breaks as the oracle's restatement of
    graph.cpp:41-195, so the orders are identical, not just equally wide."""
    m = bnpp.Model.load(model_path(name))
    rm = refcpu.Model.load(model_path(name))
    order, width = bnpp.ordering(m, {}, h)
    ro, rw = rm.ordering(list(range(rm.n_vars)), h)
    assert order == ro
    assert width == rw


def test_ordering_with_evidence_skips_evidence_vars():
    m = bnpp.Model.load(model_path("grid3x3.uai"))
    ev = evidence_of("grid3x3-PR.uai.evid")
    order, width = bnpp.ordering(m, ev, "mf")
    assert sorted(order) == sorted(v for v in range(9) if v not in ev)
    assert width >= 1


def test_plan_stats():
    m = bnpp.Model.load(model_path("ising10x10.uai"))
    st = bnpp.plan_stats(m, 0, {}, "mf")
    entries, arena, levels, buckets, width = st[:5]
    _, w = bnpp.ordering(m, {}, "mf")
    assert width == w == 13
    assert buckets >= 99 and levels >= 1 and entries > 0 and arena > 0
    st_mar = bnpp.plan_stats(m, 1, {}, "mf")
    assert st_mar[3] > 10 * buckets          # one VE per target, batched, shared buckets once
    os.environ["BNPP_NO_DEDUP"] = "1"
    try:
        st_all = bnpp.plan_stats(m, 1, {}, "mf")
    finally:
        del os.environ["BNPP_NO_DEDUP"]
    assert st_all[3] > 50 * buckets          # every target's own copy of every bucket
    assert st_all[3] > 2 * st_mar[3] and st_all[0] > st_mar[0]


def test_per_target_plans_share_identical_buckets():
    """BN::marginals runs one VE per target (model.cpp:326-334); targets whose
    min-fill orders share a prefix share those buckets exactly (same inputs,
    same layout, same level), so the schedule runs each once: 147,456 buckets
    -> about 25,000 on the 12x32 strip, same result tables per target."""
    m = bnpp.Model.load(model_path("ising12x32.uai"))
    st = bnpp.plan_stats(m, 1, {}, "mf")
    assert st[3] < 0.25 * 384 * 384


def test_bad_arguments_are_rejected():
    m = bnpp.Model.load(model_path("grid3x3.uai"))
    with pytest.raises(bnpp.BnppError) as e:
        bnpp.ordering(m, {0: 5}, "mf")      # value out of range
    assert e.value.status == bnpp.ERR_INVALID
    with pytest.raises(bnpp.BnppError) as e:
        bnpp.plan_stats(m, 7)                # unknown job kind
    assert e.value.status == bnpp.ERR_INVALID


def test_plan_stats_bucket_tree():
    """kind 3 (bucket-tree marginals) plans about three VE passes for ALL
    targets, far less than one VE per target (kind 1)."""
    m = bnpp.Model.load(model_path("ising10x10.uai"))
    pr = bnpp.plan_stats(m, 0, {}, "mf")
    tree = bnpp.plan_stats(m, 3, {}, "mf")
    per_target = bnpp.plan_stats(m, 1, {}, "mf")
    assert tree[4] == pr[4]                            # same ordering, same width
    assert pr[0] < tree[0] < 6 * pr[0]                 # factor-entries: a few passes
    assert tree[0] < per_target[0] / 10
    assert tree[7] == 1                                # one schedule
    col = [r * 10 + c for c in range(10) for r in range(10)]
    st = bnpp.plan_stats(m, 3, {}, "mf", order=col)
    assert st[4] == 10
    with pytest.raises(bnpp.BnppError) as e:           # explicit order must cover every variable
        bnpp.plan_stats(m, 3, {}, "mf", order=col[:-1])
    assert e.value.status == bnpp.ERR_INVALID


def test_bucket_tree_rejects_null_context():
    m = bnpp.Model.load(model_path("grid3x3.uai"))
    null_ctx = type("NullCtx", (), {"handle": None})()
    with pytest.raises(bnpp.BnppError) as e:
        bnpp.marginals_tree(null_ctx, m)
    assert e.value.status == bnpp.ERR_INVALID


def test_plan_stats_checkpointed_chain():
    """Column-sweep grids give chain-shaped bucket trees: with few checkpoint
    slots the plan recomputes forward messages (more entries) and runs in
    program order (one bucket per level), except the reductions of a delivered
    kept table, which sit one level after their own input and share levels
    (BNPP_NO_FREE_REDUCE=1: strictly one bucket per level)."""
    import os
    m = bnpp.Model.load(model_path("ising10x10.uai"))
    col = [r * 10 + c for c in range(10) for r in range(10)]
    full = bnpp.plan_stats(m, 3, {}, "mf", order=col)
    os.environ["BNPP_TREE_SLOTS"] = "2"
    os.environ["BNPP_NO_CHAIN"] = "1"          # one launch per bucket (fused runs add shared G products)
    try:
        ck = bnpp.plan_stats(m, 3, {}, "mf", order=col)
        os.environ["BNPP_NO_FREE_REDUCE"] = "1"
        seq = bnpp.plan_stats(m, 3, {}, "mf", order=col)
        with pytest.raises(bnpp.BnppError) as e:     # min-fill on alarm: not a chain
            bnpp.plan_stats(bnpp.Model.load(model_path("alarm.uai")), 3, {}, "mf")
        assert e.value.status == bnpp.ERR_UNSUPPORTED
    finally:
        for k in ("BNPP_TREE_SLOTS", "BNPP_NO_CHAIN", "BNPP_NO_FREE_REDUCE"):
            os.environ.pop(k, None)
    assert ck[0] > full[0]                           # recomputation
    assert seq[2] == seq[3]                          # one bucket per level
    assert ck[2] <= ck[3] and ck[3] == seq[3] and ck[0] == seq[0] and ck[6] == seq[6]
    assert ck[1] < full[1]                           # smaller arena


@pytest.mark.parametrize("n_parts", [1, 2, 3, 8])
def test_tree_parts_cover_every_marginal_once(n_parts):
    """bnpp_marginals_tree_part's ownership: every variable exactly once over
    the parts, contiguous segments of the chain for a column-sweep order, and
    per-part work well below a whole tree when the chain is split."""
    m = bnpp.Model.load(model_path("ising10x10.uai"))
    col = [r * 10 + c for c in range(10) for r in range(10)]
    seen = []
    for part in range(n_parts):
        owned, st = bnpp.plan_tree_part(m, part, n_parts, {}, order=col)
        pos = sorted(col.index(v) for v in owned)
        assert pos == list(range(pos[0], pos[0] + len(pos))) if pos else True
        seen += owned
    assert sorted(seen) == list(range(m.n_vars))
    # a non-chain tree (min-fill on alarm with evidence) is dealt round robin
    a = bnpp.Model.load(model_path("alarm.uai"))
    ev = bnpp.load_evidence(model_path("alarm.uai.evid"))
    seen = []
    for part in range(n_parts):
        seen += bnpp.plan_tree_part(a, part, n_parts, ev)[0]
    assert sorted(seen) == list(range(a.n_vars))


def test_plan_fused_sweep_cuts_traffic():
    """The 32x32 Ising bucket tree on a column sweep (width 32, checkpointed
    chain) with fused sweep runs (chain.cuh) plans the same factor-entries as
    one bucket per launch but at least 3x less algorithmic HBM traffic."""
    from bnpp import synth
    m = bnpp.Model.from_dict(synth.ising_grid(32, 32, seed=0))
    col = [r * 32 + c for c in range(32) for r in range(32)]
    os.environ["BNPP_MEM_BUDGET_GB"] = "245"
    try:
        fused = bnpp.plan_stats(m, 3, {}, "mf", dtype=bnpp.F32, order=col)
        os.environ["BNPP_NO_CHAIN"] = "1"
        plain = bnpp.plan_stats(m, 3, {}, "mf", dtype=bnpp.F32, order=col)
    finally:
        del os.environ["BNPP_MEM_BUDGET_GB"]
        os.environ.pop("BNPP_NO_CHAIN", None)
    assert fused[4] == plain[4] == 32
    assert abs(fused[0] - plain[0]) < 0.01 * plain[0]
    assert fused[6] * 3 < plain[6]


def test_plan_uses_summing_runs():
    """A tall column sweep ends in a column whose buckets only sum: the plan
    fuses them (kChainSum): less traffic than with fusion disabled."""
    from bnpp import synth
    m = bnpp.Model.from_dict(synth.ising_grid(14, 5, seed=8))
    col = [i * 5 + j for j in range(5) for i in range(14)]
    fused = bnpp.plan_stats(m, 0, {}, "mf", dtype=bnpp.F32, order=col)
    os.environ["BNPP_NO_CHAIN"] = "1"
    try:
        plain = bnpp.plan_stats(m, 0, {}, "mf", dtype=bnpp.F32, order=col)
    finally:
        del os.environ["BNPP_NO_CHAIN"]
    assert fused[6] < 0.6 * plain[6]


def _chain_forms(capfd, m, order, env, kind=0):
    """kernel forms the planner picks (BNPP_DEBUG_CHAIN lines on fd 2)."""
    old = {k: os.environ.get(k) for k in list(env) + ["BNPP_DEBUG_CHAIN"]}
    os.environ.update(env, BNPP_DEBUG_CHAIN="1")
    try:
        capfd.readouterr()
        bnpp.plan_stats(m, kind, {}, "mf", dtype=bnpp.F32, order=order)
        err = capfd.readouterr().err
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    forms = set()
    for line in err.splitlines():
        if line.startswith("[chain] run form"):
            p = line.split()
            forms.add((int(p[3]), int(p[5].split("=")[1])))      # (form, F)
    return forms


def test_plan_short_forward_runs_use_vector_form(capfd):
    """Forward runs capped at 3 buckets on a tall sweep take kChainFwdV (form 4)
    unless BNPP_NO_CHAIN_FWDV; the same runs then use the one-entry form 1."""
    from bnpp import synth
    m = bnpp.Model.from_dict(synth.ising_grid(16, 5, seed=11))
    col = [i * 5 + j for j in range(5) for i in range(16)]
    forms = _chain_forms(capfd, m, col, {"BNPP_CHAIN_RUN_MAX": "3"})
    assert (4, 3) in forms and (1, 3) not in forms, forms
    forms = _chain_forms(capfd, m, col, {"BNPP_CHAIN_RUN_MAX": "3", "BNPP_NO_CHAIN_FWDV": "1"})
    assert (1, 3) in forms and (4, 3) not in forms, forms


def test_plan_forward_runs_of_six(capfd):
    """Binary fp32 sweeps of a checkpointed bucket tree fuse 6 forward buckets
    per pass (256-B rows staged in 128-B parts) and 6 backward ones in the
    one-thread forms; with the split forms (chainsplit.cuh) runs of 7-8 --
    dense addressing (forms 7, 8) on a grid sweep, the general one (5, 6) with
    BNPP_NO_DENSE."""
    from bnpp import synth
    m = bnpp.Model.from_dict(synth.ising_grid(16, 5, seed=11))
    col = [i * 5 + j for j in range(5) for i in range(16)]
    forms = _chain_forms(capfd, m, col, {"BNPP_TREE_SLOTS": "3", "BNPP_NO_SPLIT": "1"}, kind=3)
    assert (1, 6) in forms and (2, 6) in forms, forms
    m = bnpp.Model.from_dict(synth.ising_grid(18, 5, seed=11))
    col = [i * 5 + j for j in range(5) for i in range(18)]
    forms = _chain_forms(capfd, m, col, {"BNPP_TREE_SLOTS": "3"}, kind=3)
    assert (7, 8) in forms and (8, 8) in forms, forms
    assert max(f for _, f in forms) == 8
    forms = _chain_forms(capfd, m, col, {"BNPP_TREE_SLOTS": "3", "BNPP_NO_DENSE": "1"}, kind=3)
    assert (5, 8) in forms and (6, 8) in forms, forms


def test_checkpoint_slot_memo_matches_fresh_search():
    """The bucket-tree planner remembers its checkpoint-slot search per model
    and budget bracket (capi.cpp SlotMemo): repeated and interleaved budgets in
    one process give the plans a fresh process's search gives."""
    import json
    import subprocess
    import sys
    m = bnpp.Model.load(model_path("ising10x10.uai"))
    col = [r * 10 + c for c in range(10) for r in range(10)]
    full_arena = bnpp.plan_stats(m, 3, {}, "mf", order=col)[1]
    budgets = [full_arena * f / 1e9 for f in (0.5, 0.75, 0.5, 0.95, 0.6, 0.52)]

    def stats(b):
        os.environ["BNPP_MEM_BUDGET_GB"] = repr(b)
        try:
            return list(bnpp.plan_stats(m, 3, {}, "mf", order=col))
        finally:
            del os.environ["BNPP_MEM_BUDGET_GB"]

    here = [stats(b) for b in budgets]
    code = ("import os, sys, json, bnpp\n"
            "m = bnpp.Model.load(sys.argv[1])\n"
            "col = [r * 10 + c for c in range(10) for r in range(10)]\n"
            "os.environ['BNPP_MEM_BUDGET_GB'] = sys.argv[2]\n"
            "print(json.dumps(list(bnpp.plan_stats(m, 3, {}, 'mf', order=col))))\n")
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(sys.path))
    for b, got in zip(budgets, here):
        out = subprocess.run([sys.executable, "-c", code, model_path("ising10x10.uai"), repr(b)], env=env,
                             capture_output=True, text=True, timeout=120, check=True).stdout
        assert json.loads(out.strip().splitlines()[-1]) == got
    assert here[0] == here[2] and here[0] != here[1] and here[1][1] <= budgets[1] * 1e9


def test_plan_reduces_kept_tables_hierarchically():
    """Deliveries with kept tables above 4096 entries reduce their targets
    through halves (PlanBuilder::reduce_many): fewer buckets than one
    reduction cascade per target, same traffic order of magnitude."""
    m = bnpp.Model.from_dict(synth.ising_grid(14, 8, seed=12))
    col = [i * 8 + j for j in range(8) for i in range(14)]
    os.environ.update({"BNPP_KEEP_LOG2": "13", "BNPP_TREE_SLOTS": "3"})
    try:
        many = bnpp.plan_stats(m, 3, {}, "mf", dtype=bnpp.F32, order=col)
        os.environ["BNPP_NO_REDUCE_MANY"] = "1"
        plain = bnpp.plan_stats(m, 3, {}, "mf", dtype=bnpp.F32, order=col)
    finally:
        for k in ("BNPP_KEEP_LOG2", "BNPP_TREE_SLOTS", "BNPP_NO_REDUCE_MANY"):
            os.environ.pop(k, None)
    assert many[3] < plain[3], (many[3], plain[3])
    assert many[6] <= plain[6] * 1.01


def test_plan_stats_saturate_on_infeasible_widths():
    """A min-fill order on the 32x32 grid (width 48) and on a 24x24 4-state
    Potts grid plans tables of 2^49 / 4^36 entries: sizes and byte counts
    saturate (plan.hpp kSatMax) instead of overflowing; the first plan reads as
    far beyond any device, the second fails cleanly with OOM instead of
    planning descriptors for it (tools/sanitize_check.sh runs this under UBSan)."""
    m = bnpp.Model.from_dict(synth.ising_grid(32, 32, seed=0))
    st = bnpp.plan_stats(m, 0, {}, "mf", dtype=bnpp.F64)
    assert st[4] >= 46 and st[1] > 1e15
    p = bnpp.Model.from_dict(synth.potts_grid(24, 24, k=4, seed=0))       # width 35: 4^36 entries
    with pytest.raises(bnpp.BnppError) as e:
        bnpp.plan_stats(p, 0, {}, "mf", dtype=bnpp.F32)
    assert e.value.status == bnpp.ERR_OOM


def test_plan_tree_sliced_shares_work_and_exchanges():
    """Message slicing (bnpp_plan_tree_sliced): every rank plans the same
    schedule (buckets, levels, exchanges, bytes) on 1/R of each message, so a
    rank's factor-entries fall ~1/R (below 1/R against the checkpointed one-rank
    tree: the sliced plan keeps every forward message); slice bits index the
    rank's log2(R) bits."""
    r = c = 16
    m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=0))
    col = [i * c + j for j in range(c) for i in range(r)]
    full = bnpp.plan_stats(m, 3, {}, "mf", dtype=bnpp.F32, order=col)
    per = []
    for R in (2, 4, 8):
        plans = [bnpp.plan_tree_sliced(m, k, R, order=col) for k in range(R)]
        st0 = plans[0][1]
        for sb, st in plans:
            assert st[2:4] == st0[2:4] and st[8:10] == st0[8:10]
            assert all(-1 <= b < R.bit_length() - 1 for b in sb)
        assert st0[8] > 0 and st0[9] > 0
        per.append(st0[0])
    assert per[0] < 0.6 * full[0]
    assert per[2] < per[1] < per[0]
    with pytest.raises(bnpp.BnppError):
        bnpp.plan_tree_sliced(m, 0, 3, order=col)              # not a power of two
    with pytest.raises(bnpp.BnppError):
        bnpp.plan_tree_sliced(bnpp.Model.load(model_path("alarm.uai")), 0, 2)   # not a chain


def test_plan_tree_sliced_exchange_steps(capfd):
    """Every re-slice is one all-gather of the ranks' (exponent, exp2) pairs,
    one collective and exactly one data pass: a pack (forward messages: the
    destination blocks must become the slowest -- a transpose that also scales
    to the common exponent) or, where the blocks already are the slowest and
    the received message is transposed anyway (backward messages), the raw
    block travels and the unpack scales each source block (xchg mode 2); no
    exchange keeps both passes."""
    r = c = 16
    m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=5))
    col = [i * c + j for j in range(c) for i in range(r)]
    for R in (2, 4, 8):
        os.environ["BNPP_DUMP_PLAN"] = "1"
        capfd.readouterr()
        try:
            _, st = bnpp.plan_tree_sliced(m, 0, R, order=col)
        finally:
            del os.environ["BNPP_DUMP_PLAN"]
        err = capfd.readouterr().err
        steps = {k: len(re.findall(r"xchg kind=%s " % k, err)) for k in "1234"}
        late = len(re.findall(r"xchg kind=4 mode=2 ", err))
        n = int(st[8])
        assert n > 0 and steps["1"] == n and steps["3"] == n, (R, n, steps)
        assert late > 0 and steps["4"] == late, (R, steps, late)       # every unpack scales
        assert steps["2"] + late == n, (R, n, steps, late)             # one data pass per exchange


def test_checkpoint_search_picks_a_fitting_slot_count():
    """The checkpoint-slot search (k-ary, probes planned in parallel): under
    budgets below the full tree's arena it returns exactly the plan of one
    fixed slot count (BNPP_TREE_SLOTS=s), the largest one whose need fits;
    a larger budget never gives more recomputation."""
    import os
    from bnpp import synth
    m = bnpp.Model.from_dict(synth.ising_grid(16, 16, seed=1))
    col = [r * 16 + c for c in range(16) for r in range(16)]
    full = bnpp.plan_stats(m, 3, {}, "mf", dtype=bnpp.F32, order=col)
    forced = {}
    try:
        for s in range(1, 65):
            os.environ["BNPP_TREE_SLOTS"] = str(s)
            forced[s] = bnpp.plan_stats(m, 3, {}, "mf", dtype=bnpp.F32, order=col)
    finally:
        os.environ.pop("BNPP_TREE_SLOTS", None)
    last = None
    try:
        for frac in (0.2, 0.35, 0.5, 0.7):
            os.environ["BNPP_MEM_BUDGET_GB"] = repr(full[1] * frac / 1e9)
            st = bnpp.plan_stats(m, 3, {}, "mf", dtype=bnpp.F32, order=col)
            match = [s for s, f in forced.items() if f[0] == st[0] and f[3] == st[3] and f[1] == st[1]]
            assert match, frac
            assert all(forced[s][1] > full[1] * frac * 0.8 for s in range(max(match) + 1, 65)
                       if forced[s][0] < st[0]), frac         # fewer entries only by outgrowing the budget
            if last is not None:
                assert st[0] <= last[0]
            last = st
    finally:
        os.environ.pop("BNPP_MEM_BUDGET_GB", None)


def test_plan_fuses_beliefs_and_shares_reduction_levels(capfd):
    """Host planning of the checkpointed tree (no device): with 2^8-entry kept
    sets on a 16x6 column sweep, every belief whose summed variables are the
    slots of the backward run that made its message is formed inside that run
    (kChainBel: the plan dump marks the run, the separate belief buckets and
    one read of each message are gone); on a 24x8 sweep with 2^16-entry kept
    sets (small beside its 2^24-entry messages) the kept tables' reductions
    share levels (BNPP_NO_FREE_REDUCE restores program order for them) with
    the same buckets and traffic and the arena to 0.1 %."""
    import os
    from bnpp import synth

    def stats(r, c, env):
        m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=3))
        col = [i * c + j for j in range(c) for i in range(r)]
        os.environ.update(env)
        capfd.readouterr()
        try:
            st = bnpp.plan_stats(m, 3, {}, "mf", dtype=bnpp.F32, order=col)
        finally:
            for k in env:
                del os.environ[k]
        return st, capfd.readouterr().err

    base = {"BNPP_KEEP_LOG2": "8", "BNPP_TREE_SLOTS": "3", "BNPP_DUMP_PLAN": "1"}
    fused, err_f = stats(16, 6, base)
    plain, err_p = stats(16, 6, dict(base, BNPP_NO_BEL_FUSE="1"))
    n_fused = err_f.count(" belief: ")
    assert n_fused >= 8 and err_p.count(" belief: ") == 0
    assert fused[3] == plain[3] - n_fused                # the belief buckets are gone
    assert fused[6] < plain[6]                           # one read of pi per fused belief
    # the same arena to 0.1 % (the placement by size class, plan.cpp
    # place_levels, may put the few small tables a fusion removes elsewhere)
    assert abs(fused[1] - plain[1]) <= 1e-3 * plain[1]
    base = {"BNPP_KEEP_LOG2": "16", "BNPP_TREE_SLOTS": "4"}
    free, _ = stats(24, 8, base)
    seq, _ = stats(24, 8, dict(base, BNPP_NO_FREE_REDUCE="1"))
    assert free[2] < seq[2]                              # fewer levels (launches)
    assert free[3] == seq[3] and free[6] == seq[6]       # same buckets, same traffic
    # the arena within 0.1 % (the runs ending at deliveries are sized for
    # their fused beliefs, and the shared levels move a few KiB of small
    # reductions' lifetimes)
    assert abs(free[1] - seq[1]) <= 1e-3 * seq[1]


def test_plan_slab_outer_dims(capfd):
    """Host planning (no device): a 16x16 column sweep's first-column buckets
    ([S slab][2][2], k = 1, the big input contiguous along S) take the slab form
    with the slower dims enumerated per block (plan dump `outer=4`, slab class
    8, two passes of tiles per block); BNPP_NO_SLAB_OUTER sends them back to
    the stream kernel with the same buckets, traffic and arena."""
    import os
    from bnpp import synth

    m = bnpp.Model.from_dict(synth.ising_grid(16, 16, seed=3))
    col = [i * 16 + j for j in range(16) for i in range(16)]

    def stats(env):
        os.environ.update(env)
        capfd.readouterr()
        try:
            st = bnpp.plan_stats(m, 3, {}, "mf", dtype=bnpp.F32, order=col)
        finally:
            for k in env:
                del os.environ[k]
        return st, capfd.readouterr().err

    on, err_on = stats({"BNPP_DUMP_PLAN": "1"})
    off, err_off = stats({"BNPP_DUMP_PLAN": "1", "BNPP_NO_SLAB_OUTER": "1"})
    outer = [ln for ln in err_on.splitlines() if " outer=" in ln]
    assert len(outer) >= 2 and all("bcls=8" in ln for ln in outer) and any("k=1" in ln for ln in outer), outer
    assert any(" passes=2" in ln for ln in outer), outer          # level slab blocks: two passes of tiles
    assert " outer=" not in err_off
    assert on[3] == off[3] and on[6] == off[6] and on[1] == off[1]


def test_generic_offset_width_at_4gib_boundary(tmp_path):
    """The 32-bit-offset generic kernels are chosen exactly when a view's
    reachable span fits 2^32 bytes (fp32 and fp64, plain and conditioned views,
    saturated spans): tests/cpp/o32_keys.cpp, headers only, no allocation."""
    import subprocess
    exe = str(tmp_path / "o32_keys")
    csrc = os.path.join(REPO, "bn-pp_amd", "csrc")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I" + csrc, os.path.join(REPO, "tests", "cpp", "o32_keys.cpp"),
                    "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    assert "o32 keys ok" in out.stdout


def test_two_lane_enqueue_order(tmp_path):
    """Sliced two-lane schedules are enqueued windows alternately
    (lane_order.hpp): a permutation keeping each lane's order, every wait on an
    event recorded earlier, every cross-lane data dependency kept, and without
    such dependencies lane 1's window k after lane 0's window k and lane 0's
    window k + 1 after lane 1's window k: tests/cpp/lane_order.cpp, headers only."""
    import subprocess
    exe = str(tmp_path / "lane_order")
    csrc = os.path.join(REPO, "bn-pp_amd", "csrc")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I" + csrc, os.path.join(REPO, "tests", "cpp", "lane_order.cpp"),
                    "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    assert "lane order ok" in out.stdout


def test_arena_placement_reaches_the_live_peak(capfd):
    """The fp64 32x32 column-sweep tree with four checkpoint slots holds at
    most seven 34.36-GB messages at once (240.79 GB); one best-fit arena
    placed it in 275.03 GB (small tables in freed messages' holes), the
    placement by size class (plan.cpp place_levels) in the live peak itself,
    so a 257.7-GB budget (85 % of an idle MI355X's free memory) plans four
    slots instead of three: 34.27 TB of traffic instead of 36.92."""
    import os
    from bnpp import synth
    m = bnpp.Model.from_dict(synth.ising_grid(32, 32, seed=0))
    col = [r * 32 + c for c in range(32) for r in range(32)]
    # (2^25 kept entries: the round-5 fp64 default the numbers above were taken with)
    os.environ.update({"BNPP_MEM_BUDGET_GB": "1000", "BNPP_TREE_SLOTS": "4", "BNPP_DEBUG_ARENA": "1",
                       "BNPP_KEEP_LOG2": "25"})
    try:
        capfd.readouterr()
        st = bnpp.plan_tree_part(m, 0, 1, {}, "mf", bnpp.F64, col)[1]
        err = capfd.readouterr().err
        os.environ.pop("BNPP_TREE_SLOTS")
        os.environ["BNPP_MEM_BUDGET_GB"] = "257.7"
        st_b = bnpp.plan_tree_part(m, 0, 1, {}, "mf", bnpp.F64, col)[1]
    finally:
        for k in ("BNPP_MEM_BUDGET_GB", "BNPP_TREE_SLOTS", "BNPP_DEBUG_ARENA", "BNPP_KEEP_LOG2"):
            os.environ.pop(k, None)
    line = [ln for ln in err.splitlines() if "ideal live peak" in ln][0]
    top, peak = (float(x) for x in line.replace("[bnpp] arena ", "").replace(" GB, ideal live peak", "")
                 .replace(" GB", "").split())
    assert top == peak and abs(st[1] / 1e9 - 240.79) < 0.05, line
    assert st_b[1] <= 257.7e9 and abs(st_b[6] - st[6]) < 1e9         # the budget now plans four slots
