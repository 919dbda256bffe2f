"""The multi-GPU drop-in (mirsha_multi: mirsha_hash_slices_multi,
mirsha_submit_slices_multi / wait / poll) through the C-ABI, bit-exact vs the
oracle.  On a one-GPU box device 0 is listed twice (two contexts, two streams,
two staging rings, two host packing pools on one GPU): the cut, the rebased
slice lists and the origin-order gather are the same code as on 8 GPUs."""
import numpy as np
import pytest

import oracle_py
from mirbft_amd import MirshaError, MultiEngine, SliceArrays, _lib

pytestmark = pytest.mark.gpu


def _requests(seed, n, max_slices=4, max_len=700, empty_every=7):
    """Slice lists with empty slices, empty (null-like) requests and mixed sizes."""
    rng = np.random.default_rng(seed)
    reqs = []
    for i in range(n):
        if i % empty_every == 3:
            reqs.append([])  # a request with no data
            continue
        k = int(rng.integers(1, max_slices + 1))
        sl = [rng.integers(0, 256, int(rng.integers(0, max_len)), dtype=np.uint8).tobytes() for _ in range(k)]
        if i % 11 == 5:
            sl.insert(1, b"")  # an empty slice inside a request
        reqs.append(sl)
    return reqs


def _want(reqs):
    return oracle_py.hash_messages([b"".join(r) for r in reqs])


@pytest.fixture(scope="module")
def multi():
    import torch

    torch.cuda.is_available()  # torch's HIP runtime first (see conftest.engine)
    m = MultiEngine([0, 0])
    yield m
    m.close()


@pytest.mark.parametrize("seed,n", [(1, 1), (2, 2), (3, 5000), (4, 40_000)])
def test_hash_slices_multi_bit_exact(multi, seed, n):
    reqs = _requests(seed, n)
    got = multi.hash_slices(reqs)
    assert np.array_equal(got, _want(reqs))
    cut = multi.last_cut()
    assert cut[0] == 0 and cut[-1] == n and cut == sorted(cut)


def test_cut_balances_bytes(multi):
    """Contiguous ranges of equal bytes: one device gets the few long
    requests, the other the many short ones."""
    reqs = [[b"x" * 60_000] for _ in range(40)] + [[b"y" * 100] for _ in range(24_000)]
    got = multi.hash_slices(reqs)
    assert np.array_equal(got, _want(reqs))
    cut = multi.last_cut()
    b0 = sum(len(r[0]) for r in reqs[: cut[1]])
    b1 = sum(len(r[0]) for r in reqs[cut[1]:])
    assert abs(b0 - b1) <= 60_000, (cut, b0, b1)


def test_config2_shaped_multi(multi):
    """2^17 requests of 3 slices (LE64 client, LE64 reqNo, 256-B payload: the
    state machine's request layout, state_machine.go:313-317) -- large enough
    for the pipelined staging on both contexts."""
    n, dl = 1 << 17, 256
    arena = oracle_py.gen_requests(0x6D6972626674AB02, 0, n, dl)
    base = arena.ctypes.data
    stride = 16 + dl
    ptr = np.empty(3 * n, dtype=np.uint64)
    ln = np.empty(3 * n, dtype=np.uint64)
    ptr[0::3] = base + np.arange(n, dtype=np.uint64) * stride
    ptr[1::3] = ptr[0::3] + 8
    ptr[2::3] = ptr[0::3] + 16
    ln[0::3], ln[1::3], ln[2::3] = 8, 8, dl
    sl = SliceArrays(ptr, ln, np.arange(0, 3 * n + 1, 3, dtype=np.uint32), keep=(arena,))
    got = multi.hash_slice_arrays(sl)
    want = oracle_py.hash_requests(arena, np.arange(n, dtype=np.uint64) * stride, np.full(n, stride), threads=8)
    assert np.array_equal(got, want)
    for k in range(2):
        prof = multi.host_profile(k)
        assert prof["total"] > 0


def test_async_multi_in_order(multi):
    """Six submissions (more than the 4-deep ring), waited out of order and
    polled; with and without dedup (per-range), every digest in origin order."""
    batches = [_requests(10 + i, 3000 + 500 * i) for i in range(6)]
    batches[2] = batches[2] + batches[2][:700]  # duplicates for the dedup flag
    tickets = [multi.submit_slices(b, dedup=(i % 2 == 0)) for i, b in enumerate(batches)]
    order = [3, 5, 4]  # 0-1 were retired by the ring; 2 is done once 3 is
    for i in order:
        assert np.array_equal(multi.wait(tickets[i]), _want(batches[i])), f"submission {i}"
    assert multi.poll(tickets[2])
    for i in (0, 1, 2):
        assert np.array_equal(tickets[i].out, _want(batches[i])), f"submission {i}"


def test_single_device_list_and_errors():
    m = MultiEngine([0])
    reqs = _requests(30, 2000)
    assert np.array_equal(m.hash_slices(reqs), _want(reqs))
    # a NULL slice with bytes: EINVAL, with the device-independent validation message
    sl = SliceArrays.from_requests(reqs)
    bad = sl.ptr.copy()
    bad[int(np.flatnonzero(sl.len)[-3])] = 0  # in the second device's range
    sl_bad = SliceArrays(bad, sl.len, sl.first, keep=(sl,))
    with pytest.raises(MirshaError) as e:
        m.hash_slice_arrays(sl_bad)
    assert e.value.code == _lib.MIRSHA_EINVAL
    m.close()


@pytest.mark.parametrize("n", [3, 9000])
def test_four_contexts(n):
    """Four device contexts (the cut, the rebased lists and the gather over
    more ranges than the paired tests); n = 3 leaves a range empty."""
    m = MultiEngine([0, 0, 0, 0])
    reqs = _requests(60 + n, n)
    assert np.array_equal(m.hash_slices(reqs), _want(reqs))
    cut = m.last_cut()
    assert len(cut) == 5 and cut[0] == 0 and cut[-1] == n and cut == sorted(cut)
    t = m.submit_slices(reqs)
    assert np.array_equal(m.wait(t), _want(reqs))
    m.close()


@pytest.mark.parametrize("pinned", [False, True])
def test_hash_arena_multi(multi, pinned):
    """mirsha_hash_arena_multi (the Go GPUHasherMulti's call): one arena,
    pageable or page-locked (mirsha_multi_host_alloc, portable), gapped and
    misaligned offsets, empty requests; config-2-sized so both ranges take
    the pipelined staging."""
    rng = np.random.default_rng(50 + pinned)
    n = 1 << 17
    lens = rng.integers(0, 600, n).astype(np.uint32)
    lens[::13] = 0
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + 3)
    size = int(off[-1] + lens[-1]) + 1
    src = rng.integers(0, 256, size, dtype=np.uint8)
    arena = multi.host_empty(size) if pinned else np.empty(size, dtype=np.uint8)
    arena[:] = src
    got = multi.hash_arena(arena, off, lens)
    assert np.array_equal(got, oracle_py.hash_requests(src, off, lens, threads=8))
    cut = multi.last_cut()
    assert cut[0] == 0 and cut[-1] == n and 0 < cut[1] < n


def test_async_multi_error_retires_other_ranges(multi):
    """A submission one device refuses (a NULL slice with bytes in the second
    range) fails with EINVAL after the other device's range has been
    retired; the multi context stays usable."""
    reqs = _requests(40, 6000)
    sl = SliceArrays.from_requests(reqs)
    bad = sl.ptr.copy()
    bad[int(np.flatnonzero(sl.len)[-5])] = 0
    with pytest.raises(MirshaError) as e:
        multi.submit_slices(SliceArrays(bad, sl.len, sl.first, keep=(sl,)))
    assert e.value.code == _lib.MIRSHA_EINVAL
    t = multi.submit_slices(sl)
    assert np.array_equal(multi.wait(t), _want(reqs))


def test_hash_arena_multi_cut_balances_bytes(multi):
    """The arena form cuts like the slice form: at the request
    boundary nearest to half the bytes, so the shares differ by at most one
    request."""
    lens = np.array([60_000] * 40 + [100] * 24_000, dtype=np.uint32)
    off = np.zeros(lens.size, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    src = np.random.default_rng(70).integers(0, 256, int(lens.sum()), dtype=np.uint8)
    got = multi.hash_arena(src, off, lens)
    assert np.array_equal(got, oracle_py.hash_requests(src, off, lens, threads=8))
    cut = multi.last_cut()
    b0, b1 = int(lens[: cut[1]].sum()), int(lens[cut[1]:].sum())
    assert abs(b0 - b1) <= 60_000, (cut, b0, b1)
    # the slice form cuts the same input at the same place
    multi.hash_slices([[src[int(o):int(o) + int(n)].tobytes()] for o, n in zip(off, lens)])
    assert multi.last_cut() == cut


@pytest.mark.parametrize("pinned", [False, True])
def test_submit_arena_multi_chunked(multi, pinned):
    """mirsha_submit_arena_multi, the twin of mirsha_submit_batch behind
    GPUHasherMulti's chunked HashBatch: a cycle in chunks (more than the ring
    holds), each chunk cut over both contexts, empty requests and messages
    longer than a chunk budget; bit-exact, origin order."""
    rng = np.random.default_rng(80 + pinned)
    n = 40_000
    lens = rng.integers(0, 900, n).astype(np.uint32)
    lens[::11] = 0
    lens[7_000::9_000] = 400_000
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    size = int(off[-1] + lens[-1]) + 1
    src = rng.integers(0, 256, size, dtype=np.uint8)
    arena = multi.host_empty(size) if pinned else np.empty(size, dtype=np.uint8)
    arena[:] = src
    out = multi.host_empty(32 * n).reshape(n, 32) if pinned else np.empty((n, 32), dtype=np.uint8)
    bounds = list(range(0, n, 4_000)) + [n]
    tickets = [multi.submit_arena(arena, off[a:b], lens[a:b], out=out[a:b]) for a, b in zip(bounds, bounds[1:])]
    assert len(tickets) == 10
    multi.wait(tickets[-1])
    assert np.array_equal(out, oracle_py.hash_requests(src, off, lens, threads=8))


def test_submit_arena_multi_error_retires_other_ranges(multi):
    """A failure inside ONE device's range after the other device has queued
    its own: request 5,500 lies outside the arena, which only the
    second context's validation sees.  The call fails with EINVAL, the first
    range's digests are final when it returns, and the next submission is
    bit-exact."""
    rng = np.random.default_rng(90)
    n = 6000
    lens = rng.integers(1, 500, n).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    src = rng.integers(0, 256, int(off[-1] + lens[-1]), dtype=np.uint8)
    want = oracle_py.hash_requests(src, off, lens)
    bad = off.copy()
    bad[5500] = src.size
    out = np.zeros((n, 32), dtype=np.uint8)
    with pytest.raises(MirshaError) as e:
        multi.submit_arena(src, bad, lens, out=out)
    assert e.value.code == _lib.MIRSHA_EINVAL
    cut = multi.last_cut()
    assert 0 < cut[1] <= 5500
    assert np.array_equal(out[: cut[1]], want[: cut[1]])  # the first range, retired before the call returned
    t = multi.submit_arena(src, off, lens)
    assert np.array_equal(multi.wait(t), want)
