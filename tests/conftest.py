import json
import os
import sys

import pytest

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
GOLDEN = os.path.join(REPO, "tests", "golden")
MODELS = os.path.join(GOLDEN, "models")
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the C ABI on the device)")


def model_path(name: str) -> str:
    return os.path.join(MODELS, name)


def evidence_of(name: str):
    from bnpp import synth
    return {} if name == "-" else synth.read_evidence(model_path(name))


@pytest.fixture(scope="session")
def golden_ve():
    with open(os.path.join(GOLDEN, "ve_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_kat():
    with open(os.path.join(GOLDEN, "kat_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_sp():
    with open(os.path.join(GOLDEN, "sp_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def ctx():
    import bnpp
    c = bnpp.Context(0)
    yield c
    c.close()
