"""A short run of the randomised soak (tests/soak_gpu.py) inside the GPU
suite: ~15 s of random shapes through every entry point, each checked
against the oracle; a fixed seed, so a failure names a reproducible case."""
import time

import numpy as np
import pytest

import soak_gpu

pytestmark = pytest.mark.gpu


def test_random_shapes_15s(engine):
    cases = (soak_gpu.case_host, soak_gpu.case_slices, soak_gpu.case_plan, soak_gpu.case_large,
             soak_gpu.case_chains)
    t0, k = time.time(), 0
    while time.time() - t0 < 15.0 or k < len(cases):
        seed = 23 * 1_000_003 + k
        cases[k % len(cases)](engine, np.random.default_rng(seed), seed)
        k += 1
    assert k >= len(cases)
