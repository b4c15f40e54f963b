"""Message-sliced bucket-tree marginals (bnpp_marginals_tree_sliced,
bnpp.dist.sliced_tree_marginals): R ranks (processes) on the box's
GPU over gloo, each holding 1/R of every message of a column-sweep chain and
re-slicing it between windows through the collective; the normalised sum of
their shares against the one-rank bucket tree (bnpp_marginals_tree) of the
same order.

Tolerances: inside a window a rank runs the one-rank tree's per-entry
arithmetic on its block (power-of-two rescaling is exact), but the marginal
reductions sum the slice variables last (across ranks, in fp64) instead of
first, so fp32 marginals agree to 2e-6 and fp64 ones to 1e-12.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

import bnpp
from bnpp import synth
from conftest import REPO

pytestmark = pytest.mark.gpu

WORKER = r"""
import json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "bn-pp_amd", "python"))
import torch
import torch.distributed as dist
import bnpp
from bnpp import synth, dist as bdist
rank, world, r, c, dt = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])
ev = json.loads(sys.argv[7])
ev = {int(k): v for k, v in ev.items()}
dist.init_process_group("gloo", rank=rank, world_size=world)
ctx = bnpp.Context(0)
m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=5))
col = [i * c + j for j in range(c) for i in range(r) if i * c + j not in ev]
res, st = bdist.sliced_tree_marginals(ctx, m, rank, world, dist, ev, "mf", dt, col)
# the identical call again: the planned job is relaunched (no planning)
res2, _ = bdist.sliced_tree_marginals(ctx, m, rank, world, dist, ev, "mf", dt, col)
relaunch = {"identical": res2 == res, "plan_ms": bnpp.last_timing()["plan_ms"]}
if rank == 0:
    print(json.dumps({"marg": res, "stats": st, "relaunch": relaunch}))
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


def _run_world(tmp_path, world, r, c, dtype, ev):
    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    procs = [subprocess.Popen([sys.executable, str(script), REPO, str(rk), str(world), str(r), str(c), str(dtype),
                               json.dumps({str(k): v for k, v in ev.items()})],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for rk in range(world)]
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
    return json.loads([l for l in outs[0].splitlines() if l.startswith("{")][0])


@pytest.mark.parametrize("world,r,c,dtype,ev", [
    (2, 16, 16, bnpp.F32, {}),
    (4, 16, 16, bnpp.F32, {}),
    (4, 12, 20, bnpp.F64, {220: 1, 239: 0}),   # evidence that keeps the column sweep a chain
])
def test_sliced_world_matches_one_rank_tree(ctx, tmp_path, world, r, c, dtype, ev):
    got = _run_world(tmp_path, world, r, c, dtype, ev)
    assert got["stats"]["calls"] > 0                    # the collective carried the exchanges
    assert got["relaunch"]["identical"] and got["relaunch"]["plan_ms"] == 0.0, got["relaunch"]
    m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=5))
    col = [i * c + j for j in range(c) for i in range(r) if i * c + j not in ev]
    ref, _ = bnpp.marginals_tree(ctx, m, ev, "mf", dtype, order=col)
    tol = 2e-6 if dtype == bnpp.F32 else 1e-12
    worst = 0.0
    for t, p in ref.items():
        q = got["marg"][str(t)]
        worst = max(worst, max(abs(x - y) for x, y in zip(q, p)))
    assert worst <= tol, worst


def test_sliced_loopback_runs_one_rank_share(ctx):
    """One rank's share with the one-GPU loopback collective (the timing path of
    tools/mar_sliced.py): it runs every exchange step and returns finite shares."""
    r = c = 16
    m = bnpp.Model.from_dict(synth.ising_grid(r, c, seed=5))
    col = [i * c + j for j in range(c) for i in range(r)]
    mant, exps, up = bnpp.marginals_tree_sliced(ctx, m, 0, 8, "loopback", order=col)
    assert len(mant) == r * c and up > 0
    for t, v in mant.items():
        assert all(x == x and x >= 0 for x in v), t


def test_sliced_requires_a_chain(ctx):
    m = bnpp.Model.load(os.path.join(REPO, "tests", "golden", "models", "alarm.uai"))
    with pytest.raises(bnpp.BnppError) as e:
        bnpp.marginals_tree_sliced(ctx, m, 0, 2, "loopback")
    assert e.value.status in (bnpp.ERR_UNSUPPORTED, bnpp.ERR_OOM)


def test_torch_collective_wraps_engine_buffers(ctx):
    """The RCCL path of bnpp.dist.TorchCollective hands the engine's device
    buffers to torch.distributed as uint8 tensors (CUDA array interface):
    the wrapped tensor aliases the engine's bytes both ways."""
    import ctypes as C
    import numpy as np
    import torch
    from bnpp import dist as bdist

    n = 4096
    p = C.c_void_p()
    bnpp._check(bnpp._lib.bnpp_malloc(ctx.handle, n, C.byref(p)), "malloc")
    try:
        src = (np.arange(n) % 251).astype(np.uint8)
        bnpp._check(bnpp._lib.bnpp_memcpy_h2d(ctx.handle, p.value, src.ctypes.data, n), "h2d")
        coll = bdist.TorchCollective(ctx, None, 2)
        t = coll._device(p.value, n)
        assert t.is_cuda and t.dtype == torch.uint8 and t.numel() == n
        assert t.data_ptr() == p.value
        assert np.array_equal(t.cpu().numpy(), src)
        t.fill_(7)
        torch.cuda.synchronize()
        back = np.empty(n, dtype=np.uint8)
        bnpp._check(bnpp._lib.bnpp_memcpy_d2h(ctx.handle, back.ctypes.data, p.value, n), "d2h")
        assert (back == 7).all()
    finally:
        bnpp._lib.bnpp_free(ctx.handle, p)


RCCL_WORKER = r"""
import ctypes as C, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "bn-pp_amd", "python"))
import numpy as np
import torch
import torch.distributed as dist
import bnpp
from bnpp import dist as bdist
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1)
ctx = bnpp.Context(0)
coll = bdist.TorchCollective(ctx, dist, 1, timeout_s=60)   # nccl groups + their first all-reduce
assert coll.backend == "nccl" and len(coll.pool) == coll.LANES
n = 1 << 20
ptrs = []
for _ in range(2):
    p = C.c_void_p()
    bnpp._check(bnpp._lib.bnpp_malloc(ctx.handle, n, C.byref(p)), "malloc")
    ptrs.append(p.value)
send, recv = ptrs
src = (np.arange(n) * 7 % 253).astype(np.uint8)
bnpp._check(bnpp._lib.bnpp_memcpy_h2d(ctx.handle, send, src.ctypes.data, n), "h2d")
for op in (bnpp.COLL_ALLGATHER, bnpp.COLL_ALLTOALL):
    zero = np.zeros(n, dtype=np.uint8)
    bnpp._check(bnpp._lib.bnpp_memcpy_h2d(ctx.handle, recv, zero.ctypes.data, n), "h2d")
    coll(op, send, recv, n, ctx.stream())              # RCCL on the engine's stream
    ctx.synchronize()
    back = np.empty(n, dtype=np.uint8)
    bnpp._check(bnpp._lib.bnpp_memcpy_d2h(ctx.handle, back.ctypes.data, recv, n), "d2h")
    assert np.array_equal(back, src), op
assert coll.calls == 2 and len(coll.groups) == 1
# bench.py's timer reduction over RCCL
dist.barrier()
tt = torch.tensor([3.5], device="cuda", dtype=torch.float64)
dist.all_reduce(tt, op=dist.ReduceOp.MAX)
assert float(tt[0]) == 3.5
for p in ptrs:
    bnpp._check(bnpp._lib.bnpp_free(ctx.handle, p), "free")
dist.destroy_process_group()
ctx.close()
print("rccl ok")
"""


def test_torch_collective_over_rccl_world1(tmp_path):
    """The nccl (RCCL) branch of bnpp.dist.TorchCollective on the box's one GPU:
    a one-rank nccl world creates the lanes' process groups, runs all-gather
    and all-to-all on the engine's own stream over engine buffers, and the
    bench's barrier + max-reduce -- the calls an 8-GPU run makes, minus the
    peers (a one-GPU box cannot host two RCCL ranks)."""
    script = tmp_path / "rccl_worker.py"
    script.write_text(RCCL_WORKER)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    p = subprocess.run([sys.executable, str(script), REPO], env=env, capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "rccl ok" in p.stdout
