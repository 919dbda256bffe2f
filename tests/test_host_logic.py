"""Host-side logic that needs no GPU: producer layouts, sharding, batch lists."""
import numpy as np
import pytest

from mirbft_amd import hashdata, sharding


def test_uint64_to_bytes_little_endian():
    assert hashdata.uint64_to_bytes(1) == b"\x01" + b"\x00" * 7
    assert hashdata.uint64_to_bytes(0x0102030405060708) == bytes([8, 7, 6, 5, 4, 3, 2, 1])


def test_request_layout():
    s = hashdata.request_hash_data(3, 9, b"xyz")
    assert [len(x) for x in s] == [8, 8, 3]
    assert hashdata.concat(s) == hashdata.uint64_to_bytes(3) + hashdata.uint64_to_bytes(9) + b"xyz"


def test_testengine_payload_is_17_bytes():
    p = hashdata.testengine_request_payload(2, 5)
    assert len(p) == 17 and p[8:9] == b"-"


def test_epoch_change_layout_counts():
    s = hashdata.epoch_change_hash_data(7, [(1, b"a" * 32)], [(1, 2, b"d" * 32)] * 3, [(1, 2, b"e" * 32)] * 2)
    assert len(s) == 1 + 2 * 1 + 3 * 3 + 3 * 2


def test_blocks_for_len():
    L = np.array([0, 55, 56, 119, 120, 272, 640, 4112, 16000])
    assert sharding.blocks_for_len(L).tolist() == [1, 1, 2, 2, 3, 5, 11, 65, 251]


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shard_ranges_cover_and_align(world):
    n, bs = 1 << 20, 20
    rs = sharding.shard_ranges(n, world, bs)
    assert rs[0][0] == 0 and rs[-1][1] == n
    for (a, b), (c, d) in zip(rs[:-1], rs[1:]):
        assert b == c
    for a, b in rs[:-1]:
        assert b % bs == 0
    sizes = [b - a for a, b in rs]
    assert max(sizes) - min(sizes) <= bs + 16


def test_shard_ranges_balance_by_blocks():
    lens = np.concatenate([np.full(100, 10000), np.full(900, 10)]).astype(np.uint32)
    rs = sharding.shard_ranges(1000, 2, 1, lengths=lens)
    blk = sharding.blocks_for_len(lens)
    w = [int(blk[a:b].sum()) for a, b in rs]
    assert abs(w[0] - w[1]) <= int(blk.max())


def test_batch_lists():
    idx, first = sharding.batch_lists(45, 20)
    assert first.tolist() == [0, 20, 40, 45]
    assert idx.tolist() == list(range(45))


def test_arena_windows_cover_and_bound():
    rng = np.random.default_rng(3)
    ln = rng.integers(16, 70000, 5000).astype(np.uint64)
    off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    cap = 10_000_000
    wins = sharding.arena_windows(off, ln, cap)
    assert wins[0][0] == 0 and wins[-1][1] == ln.size
    for (a0, a1, base), (b0, _, _) in zip(wins, wins[1:] + [(ln.size, None, None)]):
        assert a1 == b0 and base == off[a0]
        assert int(off[a1 - 1] + ln[a1 - 1]) - base <= cap
    order = sharding.window_orders(ln, wins)
    for i0, i1, _ in wins:
        o = order[i0:i1]
        assert sorted(o.tolist()) == list(range(i1 - i0))
        blk = sharding.blocks_for_len(ln[i0:i1][o]).astype(np.int64)
        assert np.all(np.diff(blk) <= 0)


def test_fused_lds_dma_mapping_matches_the_tile_swizzle():
    """The fused launch's LDS-DMA loader (mirsha_kernels.hip, hash_tile): lane l
    of DMA piece j lands in 16-byte slot 64 j + l of the wave's tile and must
    fetch the chunk the transposed read expects there -- message 16 j + l / 4,
    quarter (l & 3) ^ ((l >> 4) & 3) -- i.e. the inverse of lds_slot(m, q) =
    4 m + (q ^ ((m >> 2) & 3)).  Every (message, quarter) exactly once."""
    def lds_slot(m, q):
        return 4 * m + (q ^ ((m >> 2) & 3))

    seen = set()
    for j in range(4):
        for lane in range(64):
            m = 16 * j + (lane >> 2)
            q = (lane & 3) ^ ((lane >> 4) & 3)
            assert lds_slot(m, q) == 64 * j + lane
            # the kernel derives the offset from the register loader's (quarter lane & 3)
            assert 16 * q == 16 * (lane & 3) + 16 * (((lane & 3) ^ ((lane >> 4) & 3)) - (lane & 3))
            seen.add((m, q))
    assert seen == {(m, q) for m in range(64) for q in range(4)}
