"""Multi-GPU decomposition of the VE path.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm).  The
path shards without any data-path exchange:

  * MAR: BN::marginals is N independent VE runs (model.cpp:326-334).  Targets
    are dealt round-robin to ranks; each rank runs its batched schedule; ONE
    all-reduce(SUM) of a sum(card)-long fp64 vector (16 KiB at 32x32) assembles
    every marginal on every rank.
  * PR: cutset conditioning.  The k "cut" variables' joint assignments are dealt
    round-robin; each rank returns log10 Z of its conditioned sub-models; one
    all-gather of the per-assignment log10 values (8 B each) and a host
    log-sum-exp give log10 Z.
  * One huge bucket: its output is split on leading variables (a view with the
    leading variable conditioned), i.e. the same cutset trick at bucket level.
  * Sliced bucket-tree MAR (bnpp_marginals_tree_sliced): every message of a
    chain-shaped tree is split over the ranks by log2(world) binary variables
    that stay in the separators for a window of the chain; each rank computes
    1/world of every bucket, and between windows one all-to-all re-slices the
    message (sliced_tree_marginals).  This is the one path with a
    data-path exchange.

The compute is passed in as a callable so the same logic runs on the GPU
engine (bench.py) and, in the CPU tests, against the oracle over gloo.
"""
from __future__ import annotations

import itertools
import math
from typing import Callable, Dict, List, Sequence


def shard(items: Sequence[int], rank: int, world: int) -> List[int]:
    """Round-robin share of `items` for `rank`."""
    return [x for i, x in enumerate(items) if i % world == rank]


def log10_sum(logs: Sequence[float]) -> float:
    finite = [x for x in logs if x != -math.inf]
    if not finite:
        return -math.inf
    m = max(finite)
    return m + math.log10(sum(10.0 ** (x - m) for x in finite))


def assemble_marginals(n_vars: int, cards: Sequence[int], part: Dict[int, List[float]],
                       dist=None) -> Dict[int, List[float]]:
    """Every rank contributes the marginals it owns (the others read as zero);
    one all_reduce(SUM) of a sum(card)-long fp64 vector assembles them all."""
    import torch

    offs = [0]
    for c in cards:
        offs.append(offs[-1] + c)
    flat = torch.zeros(offs[-1], dtype=torch.float64)
    for t, vals in part.items():
        flat[offs[t]:offs[t] + cards[t]] = torch.tensor(vals, dtype=torch.float64)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dev = _comm_device(dist)
        buf = flat.to(dev)
        dist.all_reduce(buf, op=dist.ReduceOp.SUM)
        flat = buf.cpu()
    return {t: flat[offs[t]:offs[t + 1]].tolist() for t in range(n_vars)}


def sharded_tree_marginals(ctx, model, rank: int, world: int, dist=None, evidence=None, heuristic: str = "mf",
                           dtype=None, order=None) -> Dict[int, List[float]]:
    """Bucket-tree marginals on `world` GPUs: part `rank` of
    bnpp_marginals_tree_part (a contiguous segment of a chain-shaped tree: its
    forward prefix, the backward messages down to it, checkpointed recomputation
    inside it), then one all_reduce(SUM)."""
    import bnpp

    mine, _ = bnpp.marginals_tree(ctx, model, evidence, heuristic, bnpp.F64 if dtype is None else dtype,
                                  order=order, part=rank, n_parts=world)
    return assemble_marginals(model.n_vars, model.cards, mine, dist)


def sharded_marginals(n_vars: int, cards: Sequence[int], rank: int, world: int,
                      compute: Callable[[List[int]], Dict[int, List[float]]], dist=None) -> Dict[int, List[float]]:
    """All marginals, each rank computing its round-robin share of targets;
    assembled by one all_reduce(SUM) over a flat float64 vector."""
    mine = shard(list(range(n_vars)), rank, world)
    part = compute(mine) if mine else {}
    return assemble_marginals(n_vars, cards, part, dist if world > 1 else None)


def cutset_assignments(cut_vars: Sequence[int], cards: Sequence[int]) -> List[Dict[int, int]]:
    return [dict(zip(cut_vars, vals)) for vals in itertools.product(*[range(cards[v]) for v in cut_vars])]


def sharded_partition(cut_vars: Sequence[int], cards: Sequence[int], evidence: Dict[int, int], rank: int, world: int,
                      compute: Callable[[Dict[int, int]], float], dist=None) -> float:
    """log10 Z by cutset conditioning: Z = sum_a Z(evidence + a).  Each rank
    evaluates its round-robin share of assignments; one all_gather of log10
    values, combined with a log-sum-exp."""
    import torch

    assigns = cutset_assignments([v for v in cut_vars if v not in evidence], cards)
    n = len(assigns)
    local = torch.full((n,), -math.inf, dtype=torch.float64)
    for i in shard(list(range(n)), rank, world):
        ev = dict(evidence)
        ev.update(assigns[i])
        local[i] = compute(ev)
    if dist is not None and world > 1:
        dev = _comm_device(dist)
        bufs = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(world)]
        dist.all_gather(bufs, local.to(dev))
        stacked = torch.stack([b.cpu() for b in bufs])
        local = stacked.max(dim=0).values          # each slot filled by exactly one rank
    return log10_sum(local.tolist())


def _comm_device(dist):
    import torch

    backend = dist.get_backend()
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class TorchCollective:
    """bnpp_collective_fn over torch.distributed for a sliced run.

    nccl (RCCL over xGMI): the engine's device buffers are wrapped as uint8
    tensors (CUDA array interface) and the collective runs on the engine's
    stream (ExternalStream), so RCCL orders itself after the pack kernel and
    the next kernel after RCCL.  gloo (tests, CPU): the engine's stream is
    synchronised, the bytes staged through host memory.

    nccl process groups: one per lane of a two-front schedule (the lanes
    exchange concurrently, each on its own communicator).  They are created,
    and their communicators initialised by one tiny all-reduce, here -- before
    the engine runs -- never from inside the engine's launch loop; a lane's
    stream is bound to the next unused group at its first exchange, which
    every rank reaches in the same order.  Build one per (context, world) and
    reuse it (sliced_tree_marginals caches it on the context): groups and
    communicators live as long as it does."""

    LANES = 2

    def __init__(self, ctx, dist, world: int, timeout_s: float = 0):
        import bnpp
        self.ctx, self.dist, self.world, self.bnpp = ctx, dist, world, bnpp
        self.backend = dist.get_backend() if dist is not None and dist.is_initialized() else "gloo"
        self.calls = 0
        self.bytes_sent = 0
        self.groups = {}               # engine stream -> process group
        self.pool = []
        self.timeout_s = timeout_s
        if self.backend == "nccl":
            import datetime
            import torch
            kw = {"timeout": datetime.timedelta(seconds=timeout_s)} if timeout_s > 0 else {}
            for _ in range(self.LANES):
                g = dist.new_group(backend="nccl", **kw)
                t = torch.zeros(1, device="cuda")
                dist.all_reduce(t, group=g)          # the communicator is set up now, not mid-run
                self.pool.append(g)
            torch.cuda.synchronize()

    def reset_stats(self):
        self.calls = 0
        self.bytes_sent = 0

    def _host(self, ptr: int, nbytes: int):
        import numpy as np
        import torch
        buf = np.empty(nbytes, dtype=np.uint8)
        self.bnpp._check(self.bnpp._lib.bnpp_memcpy_d2h(self.ctx.handle, buf.ctypes.data, ptr, nbytes), "d2h")
        return torch.from_numpy(buf)

    def _device(self, ptr: int, nbytes: int):
        import torch

        class _CAI:
            pass
        o = _CAI()
        o.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 3,
                                      "strides": None}
        return torch.as_tensor(o, device="cuda")

    def __call__(self, op: int, send: int, recv: int, nbytes: int, stream: int):
        import torch
        import bnpp
        self.calls += 1
        R = self.world
        self.bytes_sent += nbytes * (R - 1)
        if self.backend == "nccl":
            if stream not in self.groups:
                if len(self.groups) >= len(self.pool):
                    raise RuntimeError("sliced run: more engine streams than prepared process groups")
                self.groups[stream] = self.pool[len(self.groups)]
            grp = self.groups[stream]
            s = torch.cuda.ExternalStream(stream)
            with torch.cuda.stream(s):
                st = self._device(send, nbytes * (R if op == bnpp.COLL_ALLTOALL else 1))
                rt = self._device(recv, nbytes * R)
                if op == bnpp.COLL_ALLGATHER:
                    self.dist.all_gather_into_tensor(rt, st, group=grp)
                else:
                    self.dist.all_to_all_single(rt, st, group=grp)
            return
        bnpp._check(bnpp._lib.bnpp_synchronize(self.ctx.handle, stream), "bnpp_synchronize")
        st = self._host(send, nbytes * (R if op == bnpp.COLL_ALLTOALL else 1))
        rt = torch.empty(nbytes * R, dtype=torch.uint8)
        if op == bnpp.COLL_ALLGATHER:
            self.dist.all_gather(list(rt.chunk(R)), st)
        else:
            self.dist.all_to_all_single(rt, st)
        arr = rt.numpy()
        bnpp._check(bnpp._lib.bnpp_memcpy_h2d(self.ctx.handle, recv, arr.ctypes.data, nbytes * R), "h2d")


def collective_for(ctx, dist, world: int, timeout_s: float = 0) -> TorchCollective:
    """The context's TorchCollective for this world (created once: its nccl
    groups and communicators are reused by every later sliced call)."""
    key = (id(dist), world, timeout_s)
    coll = getattr(ctx, "_sliced_coll", None)
    if coll is None or getattr(ctx, "_sliced_coll_key", None) != key:
        coll = TorchCollective(ctx, dist, world, timeout_s)
        ctx._sliced_coll, ctx._sliced_coll_key = coll, key
    coll.reset_stats()
    return coll


def combine_shares(n_vars: int, cards: Sequence[int], mant: Dict[int, List[float]], exps: Dict[int, int],
                   dist=None) -> Dict[int, List[float]]:
    """Sum every rank's share mantissa * 2^exp2 (one all_reduce(MAX) of the
    exponents, one all_reduce(SUM) of the aligned fp64 shares) and normalise."""
    import torch

    offs = [0]
    for c in cards:
        offs.append(offs[-1] + c)
    flat = torch.zeros(offs[-1], dtype=torch.float64)
    ex = torch.full((n_vars,), -(1 << 40), dtype=torch.int64)
    for t, e in exps.items():
        ex[t] = e
    multi = dist is not None and dist.is_initialized() and dist.get_world_size() > 1
    if multi:
        dev = _comm_device(dist)
        eb = ex.to(dev)
        dist.all_reduce(eb, op=dist.ReduceOp.MAX)
        emax = eb.cpu()
    else:
        emax = ex
    for t, vals in mant.items():
        sh = int(max(min(exps[t] - int(emax[t]), 4000), -4000))
        flat[offs[t]:offs[t] + cards[t]] = torch.tensor([math.ldexp(v, sh) for v in vals], dtype=torch.float64)
    if multi:
        buf = flat.to(_comm_device(dist))
        dist.all_reduce(buf, op=dist.ReduceOp.SUM)
        flat = buf.cpu()
    res = {}
    for t in range(n_vars):
        v = flat[offs[t]:offs[t + 1]]
        z = float(v.sum())
        res[t] = (v / z).tolist() if z > 0 else [1.0 / cards[t]] * cards[t]
    return res


def torch_min_budget_gb(dist) -> float:
    """0.85 x the smallest free device memory over the ranks, in GB (0: the
    engine's own choice, when no distributed world or no device is up)."""
    import os
    import torch
    if os.environ.get("BNPP_MEM_BUDGET_GB"):
        return float(os.environ["BNPP_MEM_BUDGET_GB"])
    if not torch.cuda.is_available():
        return 0.0
    free = torch.tensor([float(torch.cuda.mem_get_info()[0])], dtype=torch.float64)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        buf = free.to(_comm_device(dist))
        dist.all_reduce(buf, op=dist.ReduceOp.MIN)
        free = buf.cpu()
    return float(free[0]) * 0.85 / 1e9


def sliced_tree_marginals(ctx, model, rank: int, world: int, dist=None, evidence=None, heuristic: str = "mf",
                          dtype=None, order=None, timeout_s: float = 0):
    """Bucket-tree marginals with every message sliced over `world` ranks
    (bnpp_marginals_tree_sliced): -> ({var: marginal}, collective stats)."""
    import bnpp

    coll = collective_for(ctx, dist, world, timeout_s)
    if not getattr(ctx, "_sliced_trimmed", False):
        # the first sliced call on this context: what it cached for other
        # calls (e.g. a segment-scheme arena) is freed, so the budget below
        # sees it; later calls reuse the sliced job's own cached arena
        ctx.trim()
        ctx._sliced_trimmed = True
    # every rank must plan the same checkpoint count (the exchanges are
    # collectives): the smallest free memory of the world sets the budget
    budget = torch_min_budget_gb(dist)
    mant, exps, up = bnpp.marginals_tree_sliced(ctx, model, rank, world, coll, evidence, heuristic,
                                                bnpp.F32 if dtype is None else dtype, order=order, budget_gb=budget)
    res = combine_shares(model.n_vars, model.cards, mant, exps, dist)
    return res, {"calls": coll.calls, "bytes_sent": coll.bytes_sent, "uptime_ms": up}
