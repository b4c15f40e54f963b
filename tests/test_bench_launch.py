"""bench.py's N-rank launch path on CPU (no GPU): `python bench.py --gpus N`
outside a launcher starts N ranks itself (torch.distributed.run as a child
process), every rank checks the world size against --gpus, and rank 0's line
reaches stdout.  BNPP_BENCH_DRYRUN=1 stops each rank after the gloo world is up
(no engine, no device)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, REPO)


def _env(**kw):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "BNPP_BENCH_CHILD"):
        env.pop(k, None)
    env.update(kw)
    return env


def test_launcher_command():
    import bench
    cmd = bench.launcher_cmd(8, 29555, ["--gpus", "8", "--steps", "5"])
    assert cmd[:4] == [sys.executable, "-u", "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-3:] == ["--gpus", "8", "--steps", "5"][-3:] and cmd[-5].endswith("bench.py")
    a = bench.parse_args(["--gpus", "4", "--steps", "7", "--warmup", "2"])
    assert (a.gpus, a.steps, a.warmup) == (4, 7, 2)


@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_starts_n_ranks(n):
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n)],
                         env=_env(BNPP_BENCH_DRYRUN="1"), capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == rec["world_size"] == n and rec["backend"] == "gloo"


def test_world_size_mismatch_fails():
    """Under a launcher that started a different number of ranks than --gpus
    asks for, the bench refuses instead of measuring the wrong world."""
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"],
                         env=_env(BNPP_BENCH_DRYRUN="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "launcher started 1 rank" in out.stderr
