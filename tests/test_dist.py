"""Multi-process decomposition over gloo, world size 2, on CPU.

The sharding logic of bnpp.dist is exercised with the oracle as the per-rank
compute (on the GPU box bench.py / the engine supplies it): target-sharded MAR
assembled by one all_reduce, cutset-sharded PR combined by one all_gather.
"""
import math
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

from conftest import REPO, model_path


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, name, evid, cut, q):
    sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch.distributed as dist
    import refcpu
    from bnpp import dist as bdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = refcpu.Model.load(model_path(name))
    ev = refcpu.load_evidence(model_path(evid)) if evid else {}

    def mar(targets):
        return {t: m.marginal(t, ev, "mf") for t in targets}

    marg = bdist.sharded_marginals(m.n_vars, m.cards, rank, world, mar, dist)

    def pr(e):
        z, _ = m.partition(e, "mf")
        return math.log10(z) if z > 0 else -math.inf

    lz = bdist.sharded_partition(cut, m.cards, ev, rank, world, pr, dist)
    q.put((rank, marg, lz))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,evid,cut", [("grid3x3.uai", "grid3x3-MAR.uai.evid", [2, 8]),
                                           ("ising6x6.uai", None, [0, 35, 17]),
                                           ("alarm.uai", "alarm.uai.evid", [1, 5])])
def test_sharded_mar_and_cutset_pr_world2(name, evid, cut):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import refcpu

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, name, evid, cut, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m = refcpu.Model.load(model_path(name))
    ev = refcpu.load_evidence(model_path(evid)) if evid else {}
    full, _ = m.marginals(ev, "mf")
    z, _ = m.partition(ev, "mf")
    for rank, marg, lz in res:
        for t in range(m.n_vars):
            assert marg[t] == pytest.approx(full[t], abs=1e-12), (rank, t)
        assert abs(lz - math.log10(z)) <= 1e-12 * max(1.0, abs(lz))


def test_shard_and_logsum_helpers():
    sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))
    from bnpp import dist as bdist
    items = list(range(10))
    parts = [bdist.shard(items, r, 3) for r in range(3)]
    assert sorted(sum(parts, [])) == items
    assert bdist.log10_sum([0.0, 0.0]) == pytest.approx(math.log10(2))
    assert bdist.log10_sum([-math.inf, 3.0]) == 3.0
    assert bdist.log10_sum([-math.inf]) == -math.inf
    a = bdist.cutset_assignments([1, 4], [2, 3, 2, 2, 3])
    assert len(a) == 9 and a[0] == {1: 0, 4: 0}


def _tree_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch.distributed as dist
    import bnpp
    import refcpu
    from bnpp import dist as bdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    path = model_path("ising8x8.uai")
    m = bnpp.Model.load(path)
    col = [r * 8 + c for c in range(8) for r in range(8)]
    owned, _ = bnpp.plan_tree_part(m, rank, world, {}, order=col)   # the engine's ownership rule
    rm = refcpu.Model.load(path)
    mine = {t: rm.marginal(t, {}, "mf") for t in owned}            # oracle as the per-rank compute
    q.put((rank, bdist.assemble_marginals(m.n_vars, m.cards, mine, dist), owned))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_tree_part_assembly(world):
    """Chain-segment ownership of bnpp_marginals_tree_part + one all_reduce
    assemble every marginal exactly once (gloo, world size 2 and 4 -- the
    driver's scaling runs use 2, 4 and 8 ranks)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import refcpu

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tree_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full, _ = refcpu.Model.load(model_path("ising8x8.uai")).marginals({}, "mf")
    owned = sorted(sum([r[2] for r in res], []))
    assert owned == list(range(64))
    for rank, marg, _ in res:
        for t in range(64):
            assert marg[t] == pytest.approx(full[t], abs=1e-12), (rank, t)


def test_collective_is_cached_per_context():
    """bnpp.dist.collective_for: one TorchCollective per (context, world) --
    an nccl one creates its per-lane process groups (and communicators) once,
    up front, not per call or from inside the engine's launch loop -- with
    its exchange counters reset for every call."""
    from bnpp import dist as bdist

    class _Ctx:
        handle = None

    ctx = _Ctx()
    a = bdist.collective_for(ctx, None, 4)
    a.calls, a.bytes_sent = 7, 99
    b = bdist.collective_for(ctx, None, 4)
    assert b is a and (b.calls, b.bytes_sent) == (0, 0)
    assert b.backend == "gloo" and b.pool == [] and b.groups == {}
    c = bdist.collective_for(ctx, None, 8)
    assert c is not a and c.world == 8
