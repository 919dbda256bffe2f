"""BASELINE config 5 (mixed 64 B - 64 KB requests) generator: the oracle's
integer length formula against an independent Python restatement, its
distribution, and oracle digests of generated messages against hashlib."""
import hashlib

import numpy as np

import oracle_py
from mirbft_amd import sharding

SEED5 = 0x6D69726266740005
MASK = (1 << 64) - 1


def splitmix64(x):
    z = (x + 0x9E3779B97F4A7C15) & MASK
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
    return z ^ (z >> 31)


def py_data_len(seed, i):
    x = splitmix64(seed ^ i ^ 0x4C454E4754480000) >> 40
    t = 10 * x
    e, m = t >> 24, t & 0xFFFFFF
    return (64 << e) + (((64 << e) * m) >> 24)


def test_length_formula_matches_python_restatement():
    for i in list(range(300)) + [2**32 + 5, 10**8 - 1, 123456789]:
        assert oracle_py.mixed_data_len(SEED5, i) == py_data_len(SEED5, i)


def test_length_distribution_octaves():
    lens = np.array([oracle_py.mixed_data_len(SEED5, i) for i in range(20000)])
    assert lens.min() >= 64 and lens.max() < 65536
    octave = np.floor(np.log2(lens / 64)).astype(int)
    frac = np.bincount(octave, minlength=10) / lens.size
    assert np.all(np.abs(frac - 0.1) < 0.015), frac
    # mean = 96 * (2^10 - 1) / 10 = 9820.8 bytes of data per request
    assert abs(lens.mean() - 9820.8) / 9820.8 < 0.03


def test_generated_messages_hash_like_hashlib():
    ids = np.array([0, 1, 15, 16, 17, 999, 10**8 - 1, 2**40 + 3], dtype=np.uint64)
    arena, off, ln = oracle_py.gen_mixed(SEED5, ids)
    got = oracle_py.hash_requests(arena, off, ln)
    for k, i in enumerate(ids):
        i = int(i)
        dl = py_data_len(SEED5, i)
        msg = (i % 16).to_bytes(8, "little") + (i // 16).to_bytes(8, "little")
        key = splitmix64(SEED5 ^ i)
        data = b"".join(splitmix64((key + j) & MASK).to_bytes(8, "little") for j in range((dl + 7) // 8))[:dl]
        msg += data
        assert ln[k] == len(msg)
        assert bytes(arena[off[k]:off[k] + ln[k]]) == msg
        assert got[k].tobytes() == hashlib.sha256(msg).digest()


def test_world8_block_balanced_cuts_of_the_1e8_stream():
    """BASELINE config 5's 10^8-request stream cut for 8 GPUs by the
    block-balanced sharder (bench.py, tests/test_gpu_config5.py): contiguous,
    covering ranges whose compression counts are each within one request's
    compressions (a 64 KB request: 1,025) of the fair share."""
    n, world = 10**8, 8
    lens = oracle_py.mixed_lengths(SEED5, 0, n)
    assert lens.min() >= 16 + 64 and lens.max() < 16 + 65536
    cuts = sharding.shard_ranges(n, world, 1, lens)
    assert cuts[0][0] == 0 and cuts[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(cuts, cuts[1:]))
    blk = sharding.blocks_for_len(lens).astype(np.int64)
    del lens
    cum = np.concatenate([[0], np.cumsum(blk)])
    fair = cum[-1] / world
    one = int(blk.max())
    shares = [int(cum[hi] - cum[lo]) for lo, hi in cuts]
    assert max(abs(s - fair) for s in shares) <= one, (shares, fair, one)
    # every shard near 12.5 M requests (the per-GPU workload of bench.py --config 5)
    assert all(abs((hi - lo) - n // world) < 0.01 * n // world for lo, hi in cuts), cuts
