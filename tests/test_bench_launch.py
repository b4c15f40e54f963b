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


def test_reference_bound_needs_a_measured_rate():
    """No CPU baseline in the run -> no reference bound (no hard-coded rate)."""
    import bench
    rec = {"wall_ms": 2000.0, "_bound": (1024, 8.3e12, 32)}
    bench.reference_bound(rec, None)
    assert "_bound" not in rec and "reference_cpu_lower_bound_s" not in rec
    rec = {"wall_ms": 2000.0, "_bound": (1024, 8.3e12, 32)}
    bench.reference_bound(rec, 7.0e6)
    assert abs(rec["reference_cpu_lower_bound_s"] - 1024 * 8.3e12 / 7.0e6) < 1e-6
    assert abs(rec["speedup_vs_reference_lower_bound"] - rec["reference_cpu_lower_bound_s"] * 1e3 / 2000.0) < 1e-6


def _line():
    seg = {"instance": "ising32x32 all marginals", "wall_ms": 1200.0, "cold_wall_ms": 1400.0,
           "reference_cpu_lower_bound_s": 1.2e9, "speedup_vs_reference_lower_bound": 1e9,
           "reference_note": "bound", "secondary": {"instance": "ising12x12.uai"}, "check": {"ok": True},
           "sliced": {"error": "watchdog: the sliced leg did not return"}}
    return {"mar": seg, "checksum_ok": True}


def test_sliced_mar_becomes_the_headline_from_four_ranks():
    import bench
    line = _line()
    sl = {"wall_ms": 500.0, "cold_wall_ms": 800.0, "exchanges_per_call": 40, "bytes_sent_per_rank": 9.0e10,
          "max_abs_diff_vs_segment_scheme": 1e-7, "ok": True}
    bench.merge_sliced(line, sl, 8)
    head, seg = line["mar"], line["mar_segment"]
    assert head["wall_ms"] == 500.0 and head["n_gpus"] == 8 and "sliced" in head["scheme"]
    assert head["secondary"] == {"instance": "ising12x12.uai"} and "secondary" not in seg
    assert abs(head["speedup_vs_reference_lower_bound"] - 1.2e9 * 1e3 / 500.0) < 1e-3
    assert seg["wall_ms"] == 1200.0 and "sliced" not in seg and "reference_cpu_lower_bound_s" not in seg
    assert json.loads(json.dumps(line)) == line


def test_slower_sliced_leg_stays_a_subfield():
    import bench
    line = _line()
    bench.merge_sliced(line, {"wall_ms": 1300.0, "ok": True}, 4)
    assert line["mar"]["wall_ms"] == 1200.0 and line["mar"]["sliced"]["wall_ms"] == 1300.0
    assert "mar_segment" not in line


def test_failed_sliced_leg_keeps_the_segment_headline():
    import bench
    line = _line()
    bench.merge_sliced(line, {"error": "RuntimeError: boom"}, 8)
    assert line["mar"]["wall_ms"] == 1200.0 and line["mar"]["sliced"] == {"error": "RuntimeError: boom"}
    assert "mar_segment" not in line


def test_secondary_default_is_the_12x12_grid():
    import bench
    assert bench.parse_args([]).secondary == "ising12x12.uai"
    assert os.path.exists(os.path.join(REPO, "tests", "golden", "models", "ising12x12.uai"))
