"""A short run of the randomised soak (tests/soak_gpu.py) inside the GPU
suite: ~15 s of random shapes through every entry point, each checked
against the oracle; a fixed seed, so a failure names a reproducible case."""
import time

import numpy as np
import pytest

import soak_gpu

pytestmark = pytest.mark.gpu


def test_random_shapes_15s(engine):
    from mirbft_amd import MultiEngine

    multi = MultiEngine([0, 0])
    pinned = (multi.host_empty(64 << 20), multi.host_empty(32 * 20000))

    def arena(eng, rng, seed):
        soak_gpu.case_arena(eng, multi, pinned, rng, seed)

    cases = (soak_gpu.case_host, soak_gpu.case_slices, soak_gpu.case_plan, soak_gpu.case_large,
             soak_gpu.case_chains, arena)
    t0, k = time.time(), 0
    while time.time() - t0 < 15.0 or k < len(cases):
        seed = 23 * 1_000_003 + k
        cases[k % len(cases)](engine, np.random.default_rng(seed), seed)
        k += 1
    multi.close()
    assert k >= len(cases)
