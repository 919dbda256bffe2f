import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, TESTS, os.path.join(TESTS, "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950); runs through the C-ABI")


def _load(name):
    with open(os.path.join(TESTS, "golden", name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def kat():
    return _load("kat.json")


@pytest.fixture(scope="session")
def layouts():
    return _load("layouts.json")


@pytest.fixture(scope="session")
def synth_fx():
    return _load("synth.json")


@pytest.fixture(scope="session")
def engine():
    """A gfx950 engine.  No skip and no fallback: on a GPU box a missing or
    broken library must fail the gpu tests loudly."""
    from mirbft_amd import Engine

    # torch's bundled HIP runtime must initialise before the system one that
    # libmirsha uses, or torch.cuda.is_available() turns False in this process
    # (measured on the MI355X box); the device-API tests allocate through torch.
    import torch

    torch.cuda.is_available()
    e = Engine(0)
    yield e
    e.close()
