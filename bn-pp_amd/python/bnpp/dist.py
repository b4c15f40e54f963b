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
