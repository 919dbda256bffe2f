"""mirsha_submit_batch (the asynchronous arena entry behind INTEGRATION.md's
chunked GPUHasher.HashBatch) through the C-ABI, bit-exact against the oracle.

The Go binding packs one Ready() cycle into a page-locked arena chunk by chunk
and submits each chunk while the next one is packed (the loop it replaces is
processor.go:133-143).  Covered: empty requests (a request with no Data, the
zero-length message), messages larger than a chunk and chunk budgets that end
inside a message (the chunk grows to the request boundary), page-locked and
pageable arenas and digest buffers, gapped (sparse) arenas, more chunks in
flight than the 4-slot ring, interleaving with mirsha_submit_slices tickets,
and the error paths."""
import numpy as np
import pytest

import oracle_py
from mirbft_amd import MirshaError, _lib

pytestmark = pytest.mark.gpu


def _cycle(seed, n, big_every=0, big_len=0, gap=0):
    """Lengths 0..700 (every 9th request empty), optional long messages,
    optional gaps between messages; returns (src bytes, off, len)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 700, n).astype(np.uint32)
    lens[::9] = 0
    for b in (55, 56, 63, 64, 119, 120):  # padding boundaries
        lens[int(rng.integers(0, n))] = b
    if big_every:
        lens[big_every // 2::big_every] = big_len
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gap)
    size = int(off[-1] + lens[-1]) + 1
    return rng.integers(0, 256, size, dtype=np.uint8), off, lens


def _chunks(off, lens, chunk_bytes):
    """The binding's chunking: requests [lo, hi) until the chunk's bytes reach
    chunk_bytes; a chunk always ends at a request boundary."""
    n, lo, out = off.size, 0, []
    while lo < n:
        hi = lo + 1
        while hi < n and int(off[hi]) - int(off[lo]) < chunk_bytes:
            hi += 1
        out.append((lo, hi))
        lo = hi
    return out


@pytest.mark.parametrize("pinned_arena,pinned_out,gap", [(True, True, 0), (True, False, 0), (False, True, 0),
                                                         (False, False, 0), (True, True, 5)])
def test_chunked_cycle_bit_exact(engine, pinned_arena, pinned_out, gap):
    src, off, lens = _cycle(11 + gap, 30_000, big_every=5000, big_len=300_000, gap=gap)
    n = off.size
    arena = engine.host_empty(src.size) if pinned_arena else np.empty(src.size, dtype=np.uint8)
    arena[:] = src
    out = engine.host_empty(32 * n).reshape(n, 32) if pinned_out else np.empty((n, 32), dtype=np.uint8)
    chunks = _chunks(off, lens, 256 * 1024)  # 256 KiB budget: ~40 chunks, several larger than the budget
    assert len(chunks) > 8
    assert any(int(lens[lo:hi].sum()) > 256 * 1024 for lo, hi in chunks)
    tickets = [engine.submit_batch(arena, off[lo:hi], lens[lo:hi], out=out[lo:hi]) for lo, hi in chunks]
    engine.wait(tickets[-1])
    assert np.array_equal(out, oracle_py.hash_requests(src, off, lens, threads=8))


@pytest.mark.parametrize("n,budget", [(30_000, 256 * 1024), (4097, 64 * 1024), (100_003, 1 << 20)])
def test_block_chunked_cycle_bit_exact(engine, n, budget):
    """The chunks HashBatch really submits (go/gpuhash.go planChunks, ADVICE
    r5): runs of whole blocks of ceil(n / 4096) requests, and blocks larger
    than a whole budget cut at request boundaries (here the 300 KB messages'
    blocks), each chunk one mirsha_submit_batch into a page-locked arena."""
    from chunking import plan_chunks

    src, off, lens = _cycle(21 + n, n, big_every=5000, big_len=300_000)
    arena = engine.host_empty(src.size)
    arena[:] = src
    out = engine.host_empty(32 * n).reshape(n, 32)
    chunks = plan_chunks(lens, budget)
    assert chunks[-1][1] == n and any(w for *_, w in chunks)
    if budget < 300_000:
        assert any(not w for *_, w in chunks)  # split blocks present
    tickets = [engine.submit_batch(arena, off[lo:hi], lens[lo:hi], out=out[lo:hi]) for lo, hi, _ in chunks]
    engine.wait(tickets[-1])
    assert np.array_equal(out, oracle_py.hash_requests(src, off, lens, threads=8))


def test_empty_and_tiny_submissions(engine):
    src = np.frombuffer(b"abc", dtype=np.uint8).copy()
    t0 = engine.submit_batch(src, np.zeros(0, np.uint64), np.zeros(0, np.uint32))  # no requests
    t1 = engine.submit_batch(src, np.array([0, 3, 1], np.uint64), np.array([3, 0, 2], np.uint32))
    got = engine.wait(t1)
    assert engine.poll(t0)
    assert [r.tobytes().hex() for r in got] == [
        "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad",
        "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855",
        oracle_py.hash_messages([b"bc"])[0].tobytes().hex(),
    ]


def test_interleaved_with_slice_submissions(engine):
    """Arena and slice submissions share one ring and one ticket sequence:
    waiting for the last retires every earlier one, in submission order."""
    src, off, lens = _cycle(21, 9000)
    slices = [[src[int(o):int(o) + int(ln)].tobytes()] for o, ln in zip(off, lens)]
    want = oracle_py.hash_requests(src, off, lens)
    t = []
    for k in range(3):
        a, b = 3000 * k, 3000 * (k + 1)
        t.append(engine.submit_batch(src, off[a:b], lens[a:b]))
        t.append(engine.submit_slices(slices[a:b]))
    engine.wait(t[-1])
    for k in range(3):
        assert np.array_equal(t[2 * k].out, want[3000 * k:3000 * (k + 1)]), k
        assert np.array_equal(t[2 * k + 1].out, want[3000 * k:3000 * (k + 1)]), k


def test_config2_shaped_chunks_pinned(engine):
    """2^18 config-2 requests (272 B, state_machine.go:313-317 layout) in 16 MiB
    chunks from a page-locked arena into a page-locked digest buffer: the
    INTEGRATION.md HashBatch shape."""
    n, dl = 1 << 18, 256
    stride = 16 + dl
    src = oracle_py.gen_requests(0x6D69726266740002, 0, n, dl)
    arena = engine.host_empty(src.size)
    arena[:] = src
    out = engine.host_empty(32 * n).reshape(n, 32)
    off = np.arange(n, dtype=np.uint64) * stride
    lens = np.full(n, stride, dtype=np.uint32)
    tickets = [engine.submit_batch(arena, off[lo:hi], lens[lo:hi], out=out[lo:hi])
               for lo, hi in _chunks(off, lens, 16 << 20)]
    assert len(tickets) == 5
    engine.wait(tickets[-1])
    assert np.array_equal(out, oracle_py.hash_requests(src, off, lens, threads=8))


def test_errors_leave_the_ring_usable(engine):
    src, off, lens = _cycle(31, 100)
    bad = off.copy()
    bad[57] = src.size  # request 57 outside the arena
    with pytest.raises(MirshaError) as e:
        engine.submit_batch(src, bad, lens)
    assert e.value.code == _lib.MIRSHA_EINVAL
    with pytest.raises(ValueError):
        engine.submit_batch(src, off, lens[:-1])
    t = engine.submit_batch(src, off, lens)
    assert np.array_equal(engine.wait(t), oracle_py.hash_requests(src, off, lens))


def test_size_limits_rejected_before_any_read(engine):
    """MIRSHA_ERANGE for a message over MIRSHA_MAX_MESSAGE_BYTES and for a
    submission whose bytes exceed one device arena (MIRSHA_MAX_DEVICE_ARENA_BYTES):
    both are decided from off / len alone, so a small buffer declared as a
    huge arena is never read; the ring stays usable."""
    import ctypes

    lib, small = engine._lib, np.zeros(64, dtype=np.uint8)
    cases = [
        (np.array([0], dtype=np.uint64), np.array([_lib.MIRSHA_MAX_MESSAGE_BYTES + 1], dtype=np.uint32), 1 << 33),
        (np.array([0, 3 << 30], dtype=np.uint64), np.array([3 << 30, 3 << 30], dtype=np.uint32), 6 << 30),
    ]
    for off, ln, arena_len in cases:
        out = np.empty((off.size, 32), dtype=np.uint8)
        t = ctypes.c_uint64(0)
        rc = lib.mirsha_submit_batch(engine.ctx, small.ctypes.data, arena_len, off.ctypes.data, ln.ctypes.data,
                                     off.size, out.ctypes.data, ctypes.byref(t))
        assert rc == _lib.MIRSHA_ERANGE and t.value == 0
    src, off, lens = _cycle(32, 50)
    t = engine.submit_batch(src, off, lens)
    assert np.array_equal(engine.wait(t), oracle_py.hash_requests(src, off, lens))


def test_pinned_outputs_at_any_alignment(engine):
    """A page-locked digests_out is written by the kernel when 16-byte
    aligned, else by a D2H copy: both bit-exact, at offsets 0, 16 and 1 of a
    mirsha_host_alloc buffer, with a pinned and a pageable arena."""
    src, off, lens = _cycle(41, 3000, big_every=700, big_len=70_000)
    n = off.size
    want = oracle_py.hash_requests(src, off, lens, threads=8)
    pinned = engine.host_empty(src.size)
    pinned[:] = src
    for arena in (src, pinned):
        for shift in (0, 16, 1):
            buf = engine.host_empty(32 * n + 32)
            out = buf[shift:shift + 32 * n].reshape(n, 32)
            t = engine.submit_batch(arena, off, lens, out=out)
            got = engine.wait(t)
            assert np.array_equal(got, want), f"shift {shift}"
            assert np.array_equal(out, want)
