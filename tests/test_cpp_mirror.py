"""The C++ class mirror (include/bnpp/bn.hpp) and the bn/mn-compatible CLI
(bin/bnpp): compile-and-link on CPU; run on the GPU against the reference's
grid3x3 / network fixtures (models/markovnets/*.PR)."""
import os
import re
import subprocess

import pytest

from conftest import REPO, model_path

LIB = os.path.join(REPO, "bn-pp_amd", "lib")
CLI = os.path.join(REPO, "bn-pp_amd", "bin", "bnpp")


def _build_mirror_check(tmp_path):
    exe = str(tmp_path / "mirror_check")
    subprocess.run(["g++", "-std=c++17", "-O1", os.path.join(REPO, "tests", "cpp", "mirror_check.cpp"),
                    "-I" + os.path.join(REPO, "include"), "-L" + LIB, "-lbnpp", "-Wl,-rpath," + LIB, "-o", exe],
                   check=True, capture_output=True, timeout=300)
    return exe


def test_mirror_compiles_and_links(tmp_path):
    assert os.path.exists(_build_mirror_check(tmp_path))


@pytest.mark.gpu
def test_mirror_runs_on_device(tmp_path):
    exe = _build_mirror_check(tmp_path)
    r = subprocess.run([exe, os.path.dirname(model_path("grid3x3.uai"))], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "OK"


def _cli(*args):
    r = subprocess.run([CLI] + list(args), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


@pytest.mark.gpu
def test_cli_partition_matches_fixtures():
    for name, ev in (("grid3x3.uai", "grid3x3-PR.uai.evid"), ("network.uai", "network.uai.evid")):
        out = _cli(model_path(name), model_path(ev), "-pr", "-mf")
        got = float(re.search(r"Partition = ([-0-9.e+]+)", out).group(1))
        want = float(open(model_path(name + ".PR")).read().split()[-1])
        assert round(got, 4 if abs(want) < 100 else 3) == want, (name, got, want)


@pytest.mark.gpu
def test_cli_marginals_tree_equals_per_target():
    outs = []
    for flag in ("-mar", "-mar-tree"):
        out = _cli(model_path("grid3x3.uai"), model_path("grid3x3-MAR.uai.evid"), flag, "-mf")
        outs.append([l for l in out.splitlines() if "Executed" not in l])
    assert outs[0] == outs[1]
    assert any("Marginals" in l for l in outs[0])


@pytest.mark.gpu
def test_cli_sum_product_matches_reference(golden_sp):
    """`bnpp model evid -mar -sp` (bn.cpp:177-178): loopy BP marginals, evidence
    ignored as in the reference (model.cpp:313-317), printed like `bn`."""
    case = next(c for c in golden_sp["cases"] if c["model"] == "asia.uai" and c["max_iter"] == 10000)
    out = _cli(model_path("asia.uai"), model_path("asia.uai.evid"), "-mar", "-sp")
    got = [float(m) for m in re.findall(r"^\d+ : ([-0-9.e+]+)\s*$", out, re.M)]
    want = [p for v in sorted(case["marginals"], key=int) for p in case["marginals"][v]]
    assert len(got) == len(want)
    for a, b in zip(got, want):
        assert abs(a - b) < 1e-6, (a, b)
