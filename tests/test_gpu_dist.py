"""The multi-GPU decomposition (bnpp.dist) with the HIP path as
the per-rank compute: two ranks (processes) over gloo on the box's GPU, each
running the engine on its share -- the chain segment of the bucket-tree MAR
(bnpp_marginals_tree_part), its round-robin targets of the per-target MAR, its
cutset assignments of the PR -- assembled by one all_reduce / all_gather, and
compared with the one-rank result; on BASELINE config 4 (the Promedas-style
noisy-OR BN, width 22) also with the reference's own PR and MAR.  (On an 8-GPU node the same code runs one
rank per GPU over RCCL; bench.py --gpus N.)

Tolerances: the segmented tree associates no differently from the whole tree
per part, but the parts' messages are recomputed from different checkpoints,
so fp32 marginals agree to 1e-6; per-target marginals (fp64) are bit-identical;
log10 Z by cutset to 1e-12 relative (a log-sum-exp of conditioned partitions).
"""
import json
import math
import os
import socket
import subprocess
import sys

import pytest

import bnpp
from bnpp import synth
from conftest import REPO, model_path

pytestmark = pytest.mark.gpu

WORKER = r"""
import json, math, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "bn-pp_amd", "python"))
import torch
import torch.distributed as dist
import bnpp
from bnpp import synth, dist as bdist
rank, world = int(sys.argv[2]), int(sys.argv[3])
dist.init_process_group("gloo", rank=rank, world_size=world)
ctx = bnpp.Context(0)
r = c = 16
m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=3))
col = [i * c + j for j in range(c) for i in range(r)]
tree = bdist.sharded_tree_marginals(ctx, m, rank, world, dist, {}, "mf", bnpp.F32, col)
a = bnpp.Model.load(os.path.join(sys.argv[1], "tests", "golden", "models", "alarm.uai"))
ev = {1: 0, 12: 1}
per = bdist.sharded_marginals(a.n_vars, a.cards, rank, world,
                              lambda ts: bnpp.marginals(ctx, a, ev, "mf", bnpp.F64, targets=ts)[0], dist)
lz = bdist.sharded_partition([0, 35, 17], m.cards, {}, rank, world,
                             lambda e: bnpp.partition(ctx, m, e, "mf", bnpp.F64, order=col)[0], dist)
# BASELINE config 4 (noisy-OR 50 -> 80, width 22, findings observed): per-target
# MAR dealt over the ranks, bucket-tree MAR by parts, PR by cutset on diseases
models = os.path.join(sys.argv[1], "tests", "golden", "models")
c4 = bnpp.Model.load(os.path.join(models, "noisyor_50_80.uai"))
ev4 = bnpp.load_evidence(os.path.join(models, "noisyor_50_80.uai.evid"))
per4 = bdist.sharded_marginals(c4.n_vars, c4.cards, rank, world,
                               lambda ts: bnpp.marginals(ctx, c4, ev4, "mf", bnpp.F64, targets=ts)[0], dist)
tree4 = bdist.sharded_tree_marginals(ctx, c4, rank, world, dist, ev4, "mf", bnpp.F64)
lz4 = bdist.sharded_partition([0, 7, 21], c4.cards, ev4, rank, world,
                              lambda e: bnpp.partition(ctx, c4, e, "mf", bnpp.F64)[0], dist)
if rank == 0:
    print(json.dumps({"tree": tree, "per": per, "lz": lz, "per4": per4, "tree4": tree4, "lz4": lz4}))
dist.barrier()
dist.destroy_process_group()
ctx.close()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_two_ranks_hip_path_match_one_rank(ctx, tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    procs = [subprocess.Popen([sys.executable, str(script), REPO, str(rk), "2"], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for rk in range(2)]
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, e[-3000:]
        outs.append(o)
    got = json.loads([l for l in outs[0].splitlines() if l.startswith("{")][0])

    r = c = 16
    m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=3))
    col = [i * c + j for j in range(c) for i in range(r)]
    tree1, _ = bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F32, order=col)
    for t, p in tree1.items():
        for x, y in zip(got["tree"][str(t)], p):
            assert abs(x - y) <= 1e-6, (t, got["tree"][str(t)], p)
    a = bnpp.Model.load(model_path("alarm.uai"))
    per1, _ = bnpp.marginals(ctx, a, {1: 0, 12: 1}, "mf", bnpp.F64)
    for t, p in per1.items():
        assert got["per"][str(t)] == p, t
    lz1 = bnpp.partition(ctx, m, {}, "mf", bnpp.F64, order=col)[0]
    assert math.isclose(got["lz"], lz1, rel_tol=1e-12), (got["lz"], lz1)

    # config 4 against the reference's own numbers (config4_golden.json:
    # BN::partition and the per-target MAR of every disease, model.cpp:250-346)
    with open(os.path.join(REPO, "tests", "golden", "config4_golden.json")) as f:
        g = json.load(f)
    ev4 = bnpp.load_evidence(model_path(g["evidence"]))
    assert abs(got["lz4"] - g["pr"]["log10Z"]) <= 1e-12 * abs(g["pr"]["log10Z"]), (got["lz4"], g["pr"])
    for key in ("per4", "tree4"):
        for t, ref in g["marginals"].items():
            for x, y in zip(got[key][t], ref["values"]):
                assert abs(x - y) <= 1e-12, (key, t, got[key][t], ref["values"])
        for v, x in ev4.items():
            assert got[key][str(v)] == [1.0 if s == x else 0.0 for s in range(2)], (key, v)
    c4 = bnpp.Model.load(model_path(g["model"]))
    per41, _ = bnpp.marginals(ctx, c4, ev4, "mf", bnpp.F64)
    for t, p in per41.items():
        assert got["per4"][str(t)] == p, t            # the per-target VEs are the same on any rank
