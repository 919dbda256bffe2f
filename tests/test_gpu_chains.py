"""Streaming checkpoint chains on the device (mirsha_chains_*): the testengine
application's NodeState.ActiveHash (testengine/recorder.go:186-256), checked
against hashlib streaming hashers (FIPS 180-4 oracle) write for write."""
import hashlib

import numpy as np
import pytest

from mirbft_amd import CheckpointChains, MirshaError

pytestmark = pytest.mark.gpu

EMPTY = bytes.fromhex("e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855")


def test_commit_checkpoint_cycles_against_hashlib(engine):
    """64 nodes, 40 Ready() cycles: each cycle commits a random number of
    request digests to random nodes (any parity, several per node per call),
    then checkpoints a random subset (Sum, then Set = reset)."""
    rng = np.random.default_rng(7)
    n = 64
    ch = CheckpointChains(engine, n)
    ref = [hashlib.sha256() for _ in range(n)]
    for cycle in range(40):
        m = int(rng.integers(0, 300))
        digests = rng.integers(0, 256, (m, 32), dtype=np.uint8)
        chain_of = rng.integers(0, n, m).astype(np.uint32)
        ch.write(digests, chain_of)
        for d, c in zip(digests, chain_of):
            ref[c].update(d.tobytes())
        cp = np.unique(rng.integers(0, n, int(rng.integers(0, 12)))).astype(np.uint32)
        got = ch.sum(cp)
        assert [g.tobytes() for g in got] == [ref[c].digest() for c in cp], cycle
        ch.reset(cp)
        for c in cp:
            ref[c] = hashlib.sha256()
    every = np.arange(n, dtype=np.uint32)
    assert [g.tobytes() for g in ch.sum(every)] == [r.digest() for r in ref]
    ch.reset(every)
    # recorder_test.go:83: a chain with nothing committed since its reset
    assert all(g.tobytes() == EMPTY for g in ch.sum(every))
    ch.close()


def test_sum_leaves_state_and_long_runs(engine):
    ch = CheckpointChains(engine, 3)
    ref = hashlib.sha256()
    rng = np.random.default_rng(3)
    for k in (1, 1, 2, 3, 5, 8, 13, 1000, 1):
        d = rng.integers(0, 256, (k, 32), dtype=np.uint8)
        ch.write(d, np.full(k, 2, dtype=np.uint32))
        ref.update(d.tobytes())
        assert ch.sum([2, 2])[1].tobytes() == ref.digest()  # duplicate ids, repeated Sum: no state change
    assert ch.sum([0])[0].tobytes() == EMPTY  # untouched chain
    ch.write(np.zeros((0, 32), np.uint8), [])
    assert ch.sum([2])[0].tobytes() == ref.digest()
    ch.close()


def test_invalid_chain_ids_raise(engine):
    ch = CheckpointChains(engine, 4)
    with pytest.raises(MirshaError):
        ch.write(np.zeros((1, 32), np.uint8), [4])
    with pytest.raises(MirshaError):
        ch.sum([9])
    with pytest.raises(MirshaError):
        ch.reset([4])
    ch.close()


def test_uneven_absorb_one_long_one_short_chain(engine):
    """One chain gets ~1e5 digests in one call, the highest chain id gets 1
    (a short chain stored after a long one in the same wave must not
    read its index list past its own end), plus odd pending counts."""
    n = 64
    ch = CheckpointChains(engine, n)
    ref = [hashlib.sha256() for _ in range(n)]
    rng = np.random.default_rng(11)
    for m_long in (100_001, 3):
        digests = rng.integers(0, 256, (m_long + 1, 32), dtype=np.uint8)
        chain_of = np.zeros(m_long + 1, dtype=np.uint32)
        chain_of[-1] = n - 1
        ch.write(digests, chain_of)
        for d, c in zip(digests, chain_of):
            ref[c].update(d.tobytes())
    every = np.arange(n, dtype=np.uint32)
    assert [g.tobytes() for g in ch.sum(every)] == [r.digest() for r in ref]
    ch.close()
