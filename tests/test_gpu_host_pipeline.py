"""Pipelined synchronous host calls (run_pipelined in mirsha_staging.hip): calls
whose packed arena exceeds one 32 MiB staging chunk go over PCIe chunk by
chunk, each chunk's messages hashed as soon as it lands and their digests
returned while later chunks are still in flight.  Every digest must still be
the oracle's (processor.go:133-143) at its origin index, whatever the chunk
cuts, the arena's memory kind, the output buffer's memory kind, the offset
base, the length mix, or messages that straddle chunk boundaries.

Run on an MI355X:  python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
"""
import hashlib

import numpy as np
import pytest

import oracle_py
import synth
from mirbft_amd import SliceArrays, sharding

pytestmark = pytest.mark.gpu

CHUNK = 32 << 20  # kStageChunk
PIPE_MAX_LEN = 256 * 64 - 9  # kPipeMaxBlocks: longer messages take the single-shot path


def _cfg2(n, data_len=256):
    stride = 16 + data_len
    arena = synth.request_arena(synth.SEED_BASE + 2, 0, n, data_len).reshape(-1)
    return arena, np.arange(n, dtype=np.uint64) * stride, np.full(n, stride, np.uint32)


def _check(eng, arena, off, ln, idx=None, first=None, out=None, batch_out=None, min_chunks=None):
    """Digests (and list digests) vs the oracle; min_chunks: the call must
    have gone through the pipelined path with at least that many H2D chunks
    (mirsha_ctx_host_profile's chunk count; 0 = single-shot staging)."""
    if idx is None:
        got = eng.hash_batch(arena, off, ln, out=out)
        bat = None
    else:
        got, bat = eng.hash_requests_then_batches(arena, off, ln, idx, first, out=out, batch_out=batch_out)
    chunks = eng.host_profile()["chunks"]
    if min_chunks is not None:
        assert chunks >= min_chunks, f"pipelined path not taken ({chunks} chunks)"
    else:
        assert chunks == 0, f"expected single-shot staging, got {chunks} chunks"
    want = oracle_py.hash_requests(np.asarray(arena), off, ln, threads=8)
    assert np.array_equal(got, want)
    if idx is not None:
        assert np.array_equal(bat, oracle_py.batch_digests(want, idx, first))
    return got


def test_config2_full_size_pageable_and_pinned(engine):
    """BASELINE config 2 through the host API: 2^20 x 272 B (9 chunks) plus
    BatchSize-20 batch digests, from a pageable and from a pinned arena, into
    pageable and pinned result buffers, twice each (buffers reused)."""
    n = 1 << 20
    arena, off, ln = _cfg2(n)
    idx, first = sharding.batch_lists(n, 20)
    want = oracle_py.hash_requests(arena, off, ln, threads=8)
    want_bat = oracle_py.batch_digests(want, idx, first)
    pinned = engine.host_empty(arena.size)
    pinned[:] = arena
    pinned_out = engine.host_empty(32 * n).reshape(n, 32)
    for src in (arena, pinned):
        for out in (np.empty((n, 32), np.uint8), pinned_out):
            bat_out = np.empty((first.size - 1, 32), np.uint8)
            for _ in range(2):
                out[:] = 0
                req, bat = engine.hash_requests_then_batches(src, off, ln, idx, first, out=out, batch_out=bat_out)
                assert np.array_equal(req, want)
                assert np.array_equal(bat, want_bat)


def _random_lists(rng, n, n_lists, max_list, null_frac=0.1):
    sizes = rng.integers(0, max_list, n_lists)
    idx = rng.integers(0, n, int(sizes.sum())).astype(np.uint32)
    idx[rng.random(idx.size) < null_frac] = 0xFFFFFFFF
    return idx, np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)


def test_gapped_arena_pipelined_with_null_lists(engine):
    """The pipelined path's general in-order layout (kInOrder: gaps between
    messages, a shifted base, messages straddling every chunk cut, all <= 16 KiB
    so no message forces the single-shot path): the per-chunk cut search,
    offsets shipped (no device scan), and random lists with null entries
    through the lists launch behind the last chunk."""
    rng = np.random.default_rng(21)
    lens = rng.integers(0, PIPE_MAX_LEN + 1, 12000).astype(np.uint32)
    gaps = rng.integers(0, 40, lens.size).astype(np.uint64)
    off = 777 + np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])]).astype(np.uint64)
    arena = rng.integers(0, 256, int(off[-1] + lens[-1]) + 3, dtype=np.uint8)
    assert arena.size > 2 * CHUNK
    idx, first = _random_lists(rng, lens.size, 700, 40)
    _check(engine, arena, off, lens, idx, first, min_chunks=3)
    _check(engine, arena, off, lens, min_chunks=3)


def test_multi_mib_messages_single_shot(engine):
    """Messages of 5-11 MiB (longer than the pipelined path's per-message
    limit) at a shifted base take the single-shot staged path."""
    rng = np.random.default_rng(21)
    lens = rng.integers(0, 5000, 30000).astype(np.uint32)
    lens[::997] = rng.integers(5 << 20, 11 << 20, lens[::997].size)  # multi-MiB messages
    gaps = rng.integers(0, 4, lens.size).astype(np.uint64)
    off = 777 + np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])]).astype(np.uint64)
    arena = rng.integers(0, 256, int(off[-1] + lens[-1]) + 3, dtype=np.uint8)
    assert arena.size > 3 * CHUNK
    _check(engine, arena, off, lens)


def test_mixed_lengths_per_chunk_order_with_lists(engine):
    """Log-uniform lengths up to the pipelined limit (a bucket order per chunk,
    gapless: offsets rebuilt by the device scan) plus random lists with null
    entries over the request digests, through the pipelined path."""
    rng = np.random.default_rng(22)
    lens = synth.log_uniform_lengths(synth.SEED_BASE + 22, 20000, 6, 14).astype(np.uint32)
    lens = np.minimum(lens, PIPE_MAX_LEN).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
    arena = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    assert arena.size > CHUNK
    idx, first = _random_lists(rng, lens.size, 900, 30)
    _check(engine, arena, off, lens, idx, first, min_chunks=2)


def test_out_of_order_dense_arena_single_shot(engine):
    """Messages not laid out in index order take the single-shot staged path
    (no chunk cut can cover them); digests still in origin order."""
    n = 200000
    arena, off, ln = _cfg2(n)
    perm = np.random.default_rng(23).permutation(n)
    _check(engine, arena, off[perm], ln[perm])  # asserts 0 chunks


def test_pipelined_equals_single_shot(engine, monkeypatch):
    n = 300000
    arena, off, ln = _cfg2(n)
    a = engine.hash_batch(arena, off, ln)
    assert engine.host_profile()["chunks"] >= 2
    monkeypatch.setenv("MIRSHA_AB", "1")
    monkeypatch.setenv("MIRSHA_NO_PIPELINED_CALLS", "1")
    b = engine.hash_batch(arena, off, ln)
    assert engine.host_profile()["chunks"] == 0
    assert np.array_equal(a, b)
    assert np.array_equal(a, oracle_py.hash_requests(arena, off, ln, threads=8))


def test_large_slice_call(engine):
    """mirsha_hash_slices over > 3 chunks of 3-slice requests (header, data,
    empty slice), the Go side's [][]byte form."""
    rng = np.random.default_rng(24)
    n = 60000
    buf = rng.integers(0, 256, n * 2200 + 64, dtype=np.uint8)
    dl = rng.integers(0, 4096, n)
    starts = np.concatenate([[0], np.cumsum(16 + dl[:-1] + 5)]).astype(np.uint64)
    slice_off = np.empty(3 * n, np.uint64)
    slice_len = np.empty(3 * n, np.uint64)
    slice_off[0::3], slice_len[0::3] = starts, 16
    slice_off[1::3], slice_len[1::3] = starts + 16, dl
    slice_off[2::3], slice_len[2::3] = starts + 16 + dl.astype(np.uint64), 0
    assert int(slice_len.sum()) > 3 * CHUNK
    first = np.arange(0, 3 * n + 1, 3, dtype=np.uint32)
    sl = SliceArrays.from_buffer(buf, slice_off, slice_len, first)
    got = engine.hash_slice_arrays(sl)
    for i in list(range(0, n, 997)) + [n - 1]:
        s = int(starts[i])
        assert got[i].tobytes() == hashlib.sha256(buf[s:s + 16 + int(dl[i])].tobytes()).digest()
    # all of them, against the oracle over the packed form
    packed = np.concatenate([buf[int(s):int(s) + 16 + int(d)] for s, d in zip(starts, dl)])
    plen = (16 + dl).astype(np.uint32)
    poff = np.concatenate([[0], np.cumsum(plen[:-1].astype(np.uint64))]).astype(np.uint64)
    assert np.array_equal(got, oracle_py.hash_requests(packed, poff, plen, threads=8))


def test_host_profile_phases(engine):
    n = 1 << 18
    arena, off, ln = _cfg2(n)
    engine.hash_batch(arena, off, ln)
    prof = engine.host_profile()
    assert set(prof) >= {"validate", "plan", "pack", "device", "scatter"}
    assert all(v >= 0 for v in prof.values())


def test_gapless_shifted_arena_device_offsets(engine, monkeypatch):
    """Gapless requests at a nonzero base: the pipelined path ships only the
    lengths and rebuilds the offsets by a device scan; equal to shipping them
    (MIRSHA_NO_OFFSET_SCAN=1) and to the oracle.  Mixed lengths, so the
    per-chunk bucket order rides along."""
    rng = np.random.default_rng(25)
    lens = rng.integers(0, 9000, 20000).astype(np.uint32)
    off = 4096 + np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
    arena = rng.integers(0, 256, int(off[-1] + lens[-1]) + 100, dtype=np.uint8)
    assert arena.size > 2 * CHUNK
    a = _check(engine, arena, off, lens, min_chunks=2)
    monkeypatch.setenv("MIRSHA_AB", "1")
    monkeypatch.setenv("MIRSHA_NO_OFFSET_SCAN", "1")
    assert np.array_equal(engine.hash_batch(arena, off, lens), a)


def test_arena_past_4gib_pipelined_and_single_shot(engine):
    """A host arena larger than one 32-bit buffer descriptor (4 GiB): ragged
    ~8 KB requests go through the pipelined path with every chunk's kernel in
    the 64-bit-address form; then the same bytes as ~64 KB requests, longer
    than the pipelined path takes, through single-shot staging."""
    rng = np.random.default_rng(4)
    total_min = (1 << 32) + (64 << 20)
    ln = rng.integers(8000, 8193, total_min // 8000 + 1).astype(np.uint32)
    ln = ln[: int(np.searchsorted(np.cumsum(ln, dtype=np.uint64), total_min)) + 1]
    off = np.zeros(ln.size, dtype=np.uint64)
    np.cumsum(ln[:-1], dtype=np.uint64, out=off[1:])
    total = int(off[-1]) + int(ln[-1])
    assert total > (1 << 32)
    arena = np.frombuffer(rng.bytes(total), dtype=np.uint8)
    _check(engine, arena, off, ln, min_chunks=100)
    # ~64 KB requests: past the pipelined path's per-message limit
    big = np.full(total // 65000, 65000, dtype=np.uint32)
    boff = np.arange(big.size, dtype=np.uint64) * 65000
    _check(engine, arena, boff, big)
