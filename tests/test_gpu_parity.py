"""Parity of the gfx950 HIP path (through the C-ABI) with the CPU oracle and the
golden fixtures.  Bit-exact: SHA-256 is integer/byte work.

Run on an MI355X:  python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
"""
import ctypes
import hashlib
import os

import numpy as np
import pytest

import oracle_py
import synth
from mirbft_amd import (ActionResults, Actions, Engine, HashRequest, MirshaError, Processor, ProcessorWorkPool,
                        gpu_hasher, hash_batch_multi, hashdata, sharding)
from mirbft_amd import _lib
from mirbft_amd.engine import (KERNEL_LISTS, KERNEL_MSGS, VARIANT_CU, VARIANT_DIRECT, VARIANT_LDS, VARIANT_LDS_ONLY,
                               VARIANT_LOWOCC, VARIANT_PAIR)

pytestmark = pytest.mark.gpu

EMPTY = "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"


# A/B kernel forms of the tools build (tools/ab_build.sh lib, loaded through
# MIRSHA_AB_LIB with MIRSHA_AB=1) join the parametrisation when
# MIRSHA_TEST_AB_VARIANTS lists them, e.g. "12".  The product library rejects them.
_AB_VARIANTS = [int(v) for v in os.environ.get("MIRSHA_TEST_AB_VARIANTS", "").split(",") if v.strip()]


@pytest.fixture(params=[VARIANT_LDS, VARIANT_DIRECT, VARIANT_LOWOCC, VARIANT_LDS_ONLY, VARIANT_PAIR, VARIANT_CU]
                + _AB_VARIANTS,
                ids=["lds", "direct", "lowocc", "lds_only", "pair", "cu"] + [f"ab{v}" for v in _AB_VARIANTS])
def eng(engine, request):
    engine.set_variant(request.param)
    yield engine
    engine.set_variant(VARIANT_LDS)


def _hex(rows):
    return [r.tobytes().hex() for r in rows]


def test_nist_vectors(eng, kat):
    got = eng.hash_messages([v["ascii"].encode() for v in kat["nist"]] + [b"a" * 1_000_000])
    assert _hex(got) == [v["sha256"] for v in kat["nist"]] + [kat["million_a"]]


def test_boundary_lengths(eng, kat):
    vs = kat["boundary"]
    got = eng.hash_messages([synth.pattern_bytes(v["len"], v["salt"]) for v in vs])
    assert _hex(got) == [v["sha256"] for v in vs]


def test_empty_message_and_empty_call(eng):
    assert _hex(eng.hash_messages([b""])) == [EMPTY]
    assert eng.hash_messages([]).shape == (0, 32)
    assert eng.hash_batch(b"", [], []).shape == (0, 32)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_lengths_misaligned_offsets(eng, seed):
    """Any byte alignment, gaps between messages, overlapping messages."""
    rng = np.random.default_rng(seed)
    n = 3000
    lens = rng.integers(0, 2100, n).astype(np.uint32)
    gaps = rng.integers(0, 9, n).astype(np.uint64)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    off[::17] = off[::17] // 3  # some overlapping / out-of-order messages
    arena = rng.integers(0, 256, int((off + lens).max()) + 5, dtype=np.uint8)
    got = eng.hash_batch(arena, off, lens)
    want = oracle_py.hash_requests(arena, off, lens)
    assert np.array_equal(got, want)


def test_every_length_0_to_600_every_alignment(eng):
    msgs = []
    for L in range(0, 601):
        msgs.append(bytes(((j * 29 + L) & 0xFF) for j in range(L)))
    # pack with a rotating 0..3 byte shift so every (length, alignment) pair occurs
    off, arena, pos = [], bytearray(), 0
    for i, m in enumerate(msgs):
        pad = (i * 5) % 4
        arena += b"\xAA" * pad
        pos += pad
        off.append(pos)
        arena += m
        pos += len(m)
    lens = [len(m) for m in msgs]
    got = eng.hash_batch(bytes(arena), off, lens)
    assert _hex(got) == [hashlib.sha256(m).hexdigest() for m in msgs]


@pytest.mark.parametrize("shift", [0, 1, 3], ids=["aligned", "shift1", "shift3"])
def test_uniform_tiles_every_length_tail_form(eng, shift):
    """Tiles whose messages share one length: the FIPS padding after the LDS
    transpose and, when the final block holds <= 16 message bytes (or only the
    bit length), the tail-form rounds with trimmed loads.  71 messages per
    length (a full tile + a partial one), packed back to back from a base of
    `shift` bytes and ending exactly at the arena end (range-checked loads)."""
    rng = np.random.default_rng(40 + shift)
    for L in range(0, 331):
        n = 71
        arena = rng.integers(0, 256, shift + n * L, dtype=np.uint8)
        off = shift + np.arange(n, dtype=np.uint64) * L
        lens = np.full(n, L, dtype=np.uint32)
        got = eng.hash_batch(arena, off, lens)
        raw = arena.tobytes()
        want = [hashlib.sha256(raw[shift + i * L: shift + (i + 1) * L]).digest() for i in range(n)]
        assert [r.tobytes() for r in got] == want, f"length {L}"


def test_mixed_buckets_origin_order(eng):
    """Lengths spanning 1..1000 blocks go through the bucketing permutation;
    digests must still come back at their origin index."""
    lens = synth.log_uniform_lengths(synth.SEED_BASE + 5, 700, 0, 16)
    msgs = [synth.data_bytes(99, i, int(n)) for i, n in enumerate(lens)]
    got = eng.hash_messages(msgs)
    assert np.array_equal(got, oracle_py.hash_messages(msgs))


def test_loguniform_fixture(eng, synth_fx):
    fx = synth_fx["loguniform"]
    msgs = [synth.data_bytes(fx["seed"], i, n) for i, n in enumerate(fx["lengths"])]
    assert _hex(eng.hash_messages(msgs)) == fx["sha256"]


def test_large_single_message(eng):
    rng = np.random.default_rng(11)
    m = rng.integers(0, 256, (16 << 20) + 13, dtype=np.uint8).tobytes()
    assert eng.hash_messages([m])[0].tobytes() == hashlib.sha256(m).digest()


def test_messages_past_2_pow_29_bytes(engine):
    """Bit lengths of 2^32 and more: the length block's high word (L >> 29)
    is nonzero only for messages of 512 MiB and up.  Two such messages (high
    word 1 with a zero low word, and with a nonzero one) beside short ones in
    one call; each is an 8.4 M-compression chain in one lane (~15-20 s)."""
    rng = np.random.default_rng(29)
    lens = [100, 1 << 29, 55, (1 << 29) + 4097, 0]
    arena = np.frombuffer(rng.bytes(sum(lens)), dtype=np.uint8)
    off = np.zeros(len(lens), dtype=np.uint64)
    np.cumsum(np.array(lens[:-1], dtype=np.uint64), out=off[1:])
    got = engine.hash_batch(arena, off, np.array(lens, dtype=np.uint32))
    mv = memoryview(arena)
    for i, L in enumerate(lens):
        o = int(off[i])
        assert got[i].tobytes() == hashlib.sha256(mv[o:o + L]).digest(), f"message {i} ({L} bytes)"


def test_testengine_requests(eng, layouts):
    rs = layouts["testengine_requests"]
    reqs = [hashdata.request_hash_data(r["client"], r["req_no"],
                                       hashdata.testengine_request_payload(r["client"], r["req_no"])) for r in rs]
    got = eng.hash_slices(reqs)
    assert _hex(got) == [r["sha256"] for r in rs]


def _digest_table(layouts):
    keys = {(r["client"], r["req_no"]): i for i, r in enumerate(layouts["testengine_requests"])}
    dig = np.frombuffer(b"".join(bytes.fromhex(r["sha256"]) for r in layouts["testengine_requests"]),
                        dtype=np.uint8).reshape(-1, 32)
    return keys, dig


def test_batches_with_null_requests(engine, layouts):
    keys, dig = _digest_table(layouts)
    idx, first = [], [0]
    for b in layouts["batches"]:
        idx += [_lib.MIRSHA_NULL_INDEX if e is None else keys[(e[0], e[1])] for e in b["entries"]]
        first.append(len(idx))
    got = engine.digest_lists(dig, idx, first)
    assert _hex(got) == [b["sha256"] for b in layouts["batches"]]


def test_batch_slices_equal_digest_lists(engine, layouts):
    """The same batches fed as [][]byte HashRequest.Data (sequence.go:154-157)."""
    keys, dig = _digest_table(layouts)
    reqs = []
    for b in layouts["batches"]:
        reqs.append(hashdata.batch_hash_data([b"" if e is None else dig[keys[(e[0], e[1])]].tobytes()
                                              for e in b["entries"]]))
    assert _hex(engine.hash_slices(reqs)) == [b["sha256"] for b in layouts["batches"]]


def test_checkpoint_chain(engine, layouts):
    keys, dig = _digest_table(layouts)
    cc = layouts["checkpoint_chain"]
    commits = [keys[(c, r)] for c, r in cc["commits"]]
    idx, first, want, start = [], [0], [], 0
    for cp in cc["checkpoints"]:
        idx += commits[start:cp["after_commit"]]
        first.append(len(idx))
        want.append(cp.get("sha256") or cp.get("empty_after_reset"))
        start = cp["after_commit"]
    assert _hex(engine.digest_lists(dig, idx, first)) == want
    assert want[-1] == EMPTY  # testengine/recorder_test.go:83


def test_epoch_change(engine, layouts):
    ec = layouts["epoch_change"]
    slices = hashdata.epoch_change_hash_data(
        ec["new_epoch"], [(s, bytes.fromhex(v)) for s, v in ec["checkpoints"]],
        [(e, s, bytes.fromhex(d)) for e, s, d in ec["p_set"]], [(e, s, bytes.fromhex(d)) for e, s, d in ec["q_set"]])
    assert _hex(engine.hash_slices([slices] * 3)) == [ec["sha256"]] * 3


def test_slices_with_empty_slices_and_requests(engine):
    reqs = [[], [b""], [b"", b"", b"abc"], [b"ab", b"", b"c"], [b"x" * 63, b"y"], [b"q" * 1000] * 5]
    want = [hashlib.sha256(b"".join(r)).hexdigest() for r in reqs]
    assert _hex(engine.hash_slices(reqs)) == want


def test_cfg2_prefix_requests_then_batches(eng, synth_fx):
    fx = synth_fx["cfg2_prefix"]
    n, bs = fx["count"], fx["batch_size"]
    arena = synth.request_arena(synth.SEED_BASE + 2, 0, n, 256)
    idx, first = sharding.batch_lists(n, bs)
    req, bat = eng.hash_requests_then_batches(arena, np.arange(n) * 272, np.full(n, 272), idx, first)
    assert hashlib.sha256(req.tobytes()).hexdigest() == fx["request_sha256_of_concat"]
    assert _hex(bat) == fx["batch_sha256"]


def test_requests_then_batches_random_with_nulls(eng):
    rng = np.random.default_rng(5)
    n = 5000
    lens = rng.integers(0, 700, n).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(lens[:-1], out=off[1:])
    arena = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    sizes = rng.integers(0, 40, 400)
    idx = rng.integers(0, n, int(sizes.sum())).astype(np.uint32)
    idx[rng.random(idx.size) < 0.1] = _lib.MIRSHA_NULL_INDEX
    first = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    req, bat = eng.hash_requests_then_batches(arena, off, lens, idx, first)
    want_req = oracle_py.hash_requests(arena, off, lens)
    assert np.array_equal(req, want_req)
    assert np.array_equal(bat, oracle_py.batch_digests(want_req, idx, first))


def test_pinned_host_arena(engine, synth_fx):
    """An arena in mirsha_host_alloc memory (the Go side's reused C arena)
    gives the same digests as a pageable one."""
    fx = synth_fx["cfg2_prefix"]
    n, bs = fx["count"], fx["batch_size"]
    src = synth.request_arena(synth.SEED_BASE + 2, 0, n, 256).reshape(-1)
    arena = engine.host_empty(src.size)
    arena[:] = src
    idx, first = sharding.batch_lists(n, bs)
    req_buf = np.zeros((n, 32), np.uint8)
    bat_buf = np.zeros((len(first) - 1, 32), np.uint8)
    for _ in range(2):  # result buffers reused across calls
        req, bat = engine.hash_requests_then_batches(arena, np.arange(n) * 272, np.full(n, 272), idx, first,
                                                     out=req_buf, batch_out=bat_buf)
        assert req is req_buf and bat is bat_buf
        assert hashlib.sha256(req.tobytes()).hexdigest() == fx["request_sha256_of_concat"]
        assert _hex(bat) == fx["batch_sha256"]
    assert engine.host_empty(0).size == 0
    with pytest.raises(ValueError):
        engine.hash_batch(arena, [0], [272], out=np.zeros((2, 32), np.uint8))


def test_invalid_arguments_raise(engine):
    with pytest.raises(MirshaError):
        engine.hash_batch(b"abc", [2], [5])  # past the arena end
    with pytest.raises(MirshaError):
        engine.digest_lists(np.zeros((2, 32), np.uint8), [0, 5], [0, 2])  # idx out of range
    with pytest.raises(MirshaError):
        engine.digest_lists(np.zeros((2, 32), np.uint8), [0, 1], [1, 2])  # first[0] != 0
    # the context is still usable afterwards
    assert _hex(engine.hash_messages([b""])) == [EMPTY]


def test_processor_mirror_origin_order(engine):
    reqs = [HashRequest(data=hashdata.request_hash_data(c, r, b"payload-%d" % (c * 7 + r)), origin=("req", c, r))
            for c in range(3) for r in range(50)]
    reqs += [HashRequest(data=hashdata.batch_hash_data([b"\x01" * 32] * k), origin=("batch", k)) for k in (1, 20, 0)]
    res = Processor(engine).process(Actions(hash=reqs))
    assert isinstance(res, ActionResults) and len(res.digests) == len(reqs)
    for hr, req in zip(res.digests, reqs):
        assert hr.request is req
        assert hr.digest == hashlib.sha256(hashdata.concat(req.data)).digest()
    pool = ProcessorWorkPool(engine, hash_workers=8)
    res2 = pool.process(Actions(hash=reqs))
    assert [r.digest for r in res2.digests] == [r.digest for r in res.digests]
    assert Processor(engine).process(Actions()).digests == []


def test_streaming_hasher(engine):
    h = gpu_hasher(engine)()
    for part in (b"ab", b"", b"c"):
        h.write(part)
    assert h.sum().hex() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    h.reset()
    assert h.sum().hex() == EMPTY


def test_cpp_host_mirror():
    host = ctypes.CDLL(_lib.HOST_LIB_PATH)
    msgs = [b"", b"abc", b"z" * 1000]
    bufs = [ctypes.create_string_buffer(m, len(m) or 1) for m in msgs]
    ptrs = (ctypes.c_void_p * 3)(*[ctypes.addressof(b) for b in bufs])
    lens = (ctypes.c_uint64 * 3)(*[len(m) for m in msgs])
    out = (ctypes.c_uint8 * 96)()
    err = ctypes.create_string_buffer(256)
    rc = host.mirbft_host_process(0, ptrs, lens, 3, out, err, 256)
    assert rc == 0, err.value
    assert [bytes(out[32 * i:32 * i + 32]) for i in range(3)] == [hashlib.sha256(m).digest() for m in msgs]


def test_multi_device_sharding_in_process(engine):
    """mirsha_hash_batch_multi on [0, 0]: two contexts, contiguous ranges, host gather."""
    rng = np.random.default_rng(3)
    n = 4001
    lens = rng.integers(0, 900, n).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(lens[:-1], out=off[1:])
    arena = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    got = hash_batch_multi([0, 0], arena, off, lens)
    assert np.array_equal(got, oracle_py.hash_requests(arena, off, lens))


# ---------------------------------------------------------------- device API


def _torch():
    import torch

    assert torch.cuda.is_available()
    return torch


def test_device_generator_matches_oracle(engine):
    torch = _torch()
    for data_len, first, count in ((256, 0, 300), (4096, 1 << 17, 40), (17, 5, 9), (0, 3, 4)):
        d = torch.empty(count * (16 + data_len), dtype=torch.uint8, device="cuda")
        engine.synth_requests_device(synth.SEED_BASE + 2, first, count, data_len, d.data_ptr())
        engine.sync()
        want = oracle_py.gen_requests(synth.SEED_BASE + 2, first, count, data_len)
        assert np.array_equal(d.cpu().numpy(), want), (data_len, first)


@pytest.mark.parametrize("cfg,data_len,n,bs", [(2, 256, 1 << 20, 20), (3, 4096, 1 << 18, 500)])
def test_full_size_configs_device_resident(engine, cfg, data_len, n, bs):
    """BASELINE configs 2 and 3 at full size, device-resident, bit-exact vs the
    oracle (multi-threaded CPU), plus the dependent batch pass."""
    torch = _torch()
    stride = 16 + data_len
    seed = synth.SEED_BASE + cfg
    d_arena = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    d_off = torch.arange(n, dtype=torch.int64, device="cuda") * stride
    d_len = torch.full((n,), stride, dtype=torch.int32, device="cuda")
    d_req = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    idx, first = sharding.batch_lists(n, bs)
    d_idx = torch.from_numpy(idx.astype(np.int32)).cuda()
    d_first = torch.from_numpy(first.astype(np.int32)).cuda()
    nb = first.size - 1
    d_bat = torch.empty((nb, 32), dtype=torch.uint8, device="cuda")
    engine.synth_requests_device(seed, 0, n, data_len, d_arena.data_ptr())
    engine.hash_batch_device(d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(), d_len.data_ptr(), None, n,
                             d_req.data_ptr())
    engine.digest_lists_device(d_req.data_ptr(), n, d_idx.data_ptr(), d_first.data_ptr(), nb, int(first[-1]),
                               d_bat.data_ptr())
    engine.sync()
    arena = oracle_py.gen_requests(seed, 0, n, data_len)
    want_req = oracle_py.hash_requests(arena, np.arange(n, dtype=np.uint64) * stride, np.full(n, stride), threads=8)
    got_req = d_req.cpu().numpy()
    assert np.array_equal(got_req, want_req)
    assert np.array_equal(d_bat.cpu().numpy(), oracle_py.batch_digests(want_req, idx, first))


def test_external_stream_and_timing(engine):
    torch = _torch()
    s = torch.cuda.Stream()
    n, data_len = 4096, 256
    d_arena = torch.empty(n * 272, dtype=torch.uint8, device="cuda")
    d_off = torch.arange(n, dtype=torch.int64, device="cuda") * 272
    d_len = torch.full((n,), 272, dtype=torch.int32, device="cuda")
    d_out = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    engine.set_stream(s.cuda_stream)
    engine.set_timing(True)
    engine.reset_timing()
    try:
        engine.synth_requests_device(7, 0, n, data_len, d_arena.data_ptr())
        for _ in range(3):
            engine.hash_batch_device(d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(), d_len.data_ptr(), None, n,
                                     d_out.data_ptr())
        s.synchronize()
        launches, ms = engine.kernel_time(KERNEL_MSGS)
        assert launches == 3 and ms > 0
        assert engine.kernel_time(KERNEL_LISTS)[0] == 0
    finally:
        engine.set_timing(False)
        engine.set_stream(None)
    want = oracle_py.hash_requests(oracle_py.gen_requests(7, 0, n, data_len), np.arange(n) * 272, np.full(n, 272))
    assert np.array_equal(d_out.cpu().numpy(), want)


def test_device_order_permutation(engine):
    torch = _torch()
    rng = np.random.default_rng(8)
    n = 3000
    lens = rng.integers(0, 3000, n).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(lens[:-1], out=off[1:])
    arena = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    from mirbft_amd import bucket_order

    order, _ = bucket_order(lens)
    d_arena = torch.from_numpy(arena).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.from_numpy(lens.view(np.int32)).cuda()
    d_order = torch.from_numpy(order.view(np.int32)).cuda()
    d_out = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    engine.hash_batch_device(d_arena.data_ptr(), arena.size, d_off.data_ptr(), d_len.data_ptr(), d_order.data_ptr(), n,
                             d_out.data_ptr())
    engine.sync()
    assert np.array_equal(d_out.cpu().numpy(), oracle_py.hash_requests(arena, off, lens))


def test_device_lists_with_nulls_and_empty(engine):
    """Device digest-list API: null entries (compaction path), empty lists, odd/even counts."""
    torch = _torch()
    rng = np.random.default_rng(12)
    nd = 777
    dig = rng.integers(0, 256, (nd, 32), dtype=np.uint8)
    sizes = rng.integers(0, 45, 1500)
    sizes[::7] = 0
    idx = rng.integers(0, nd, int(sizes.sum())).astype(np.uint32)
    idx[rng.random(idx.size) < 0.15] = _lib.MIRSHA_NULL_INDEX
    first = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    d_dig = torch.from_numpy(dig).cuda()
    d_idx = torch.from_numpy(idx.view(np.int32)).cuda()
    d_first = torch.from_numpy(first.view(np.int32)).cuda()
    d_out = torch.empty((sizes.size, 32), dtype=torch.uint8, device="cuda")
    engine.digest_lists_device(d_dig.data_ptr(), nd, d_idx.data_ptr(), d_first.data_ptr(), sizes.size,
                               int(first[-1]), d_out.data_ptr())
    engine.sync()
    assert np.array_equal(d_out.cpu().numpy(), oracle_py.batch_digests(dig, idx, first))


def _plan_run(engine, plan, arena, off, lens, n_lists, runs=2):
    """Runs a plan `runs` times on device copies of (arena, off, lens); returns (req, lists)."""
    torch = _torch()
    n = lens.size
    d_arena = torch.from_numpy(np.ascontiguousarray(arena)).cuda()
    d_off = torch.from_numpy(np.ascontiguousarray(off, dtype=np.uint64).view(np.int64)).cuda()
    d_len = torch.from_numpy(np.ascontiguousarray(lens, dtype=np.uint32).view(np.int32)).cuda()
    d_req = torch.empty((max(n, 1), 32), dtype=torch.uint8, device="cuda")
    d_lst = torch.empty((max(n_lists, 1), 32), dtype=torch.uint8, device="cuda")
    out = []
    for _ in range(runs):
        d_req.zero_()
        d_lst.zero_()
        torch.cuda.synchronize()  # torch's stream vs the engine's own (non-blocking) stream
        engine.hash_requests_then_batches_device(plan, d_arena.data_ptr(), arena.size, d_off.data_ptr(),
                                                 d_len.data_ptr(), d_req.data_ptr(), d_lst.data_ptr())
        plan.status()
        out.append((d_req.cpu().numpy()[:n].copy(), d_lst.cpu().numpy()[:n_lists].copy()))
    return out


@pytest.mark.parametrize("mode", ["auto", "fused", "sequential"])
@pytest.mark.parametrize("cfg,data_len,n,bs", [(2, 256, 1 << 20, 20), (3, 4096, 1 << 18, 500), (9, 100, 5003, 7)])
def test_pipeline_device_full_size(engine, mode, cfg, data_len, n, bs):
    """Request -> batch digests through a plan at BASELINE sizes (fused: one
    persistent launch with readiness counters), bit-exact vs the oracle, run
    twice on the same plan (tickets / counters carried across runs)."""
    torch = _torch()
    stride = 16 + data_len
    seed = synth.SEED_BASE + cfg
    idx, first = sharding.batch_lists(n, bs)
    plan = engine.pipeline(n, idx, first, np.full(n, stride), mode=mode)
    if mode == "auto":  # long VerifyBatch chains -> fused launch; short batches -> two kernels
        assert plan.mode_name == ("fused" if bs == 500 else "sequential")
    else:
        assert plan.mode_name == mode
    if plan.mode_name == "fused" and cfg == 3:  # 4,096 tiles > the tile-wave slots: split tiles
        assert plan.split_tiles()[0] > 0
    d_arena = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    d_off = torch.arange(n, dtype=torch.int64, device="cuda") * stride
    d_len = torch.full((n,), stride, dtype=torch.int32, device="cuda")
    d_req = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    d_bat = torch.empty((first.size - 1, 32), dtype=torch.uint8, device="cuda")
    engine.synth_requests_device(seed, 0, n, data_len, d_arena.data_ptr())
    arena = oracle_py.gen_requests(seed, 0, n, data_len)
    want_req = oracle_py.hash_requests(arena, np.arange(n, dtype=np.uint64) * stride, np.full(n, stride), threads=8)
    want_bat = oracle_py.batch_digests(want_req, idx, first)
    for _ in range(2):
        d_req.zero_()
        d_bat.zero_()
        torch.cuda.synchronize()  # torch's stream vs the engine's own (non-blocking) stream
        engine.hash_requests_then_batches_device(plan, d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(),
                                                 d_len.data_ptr(), d_req.data_ptr(), d_bat.data_ptr())
        plan.status()
        assert np.array_equal(d_req.cpu().numpy(), want_req)
        assert np.array_equal(d_bat.cpu().numpy(), want_bat)
    plan.close()


@pytest.mark.parametrize("mode,data_len,bs,n,cycles", [
    ("sequential", 256, 20, 50_003, 3), ("sequential", 256, 20, 1 << 20, 2),
    ("fused", 4096, 500, 16_411, 3), ("fused", 4096, 500, 1 << 18, 2)])
def test_pipeline_overlap_cycles(engine, mode, data_len, bs, n, cycles):
    """Overlapped cycles (mirsha_pipeline_overlap_device): each launch hashes
    cycle i's requests and cycle i-1's batch digests (BatchSize 20 on a
    sequential plan, VerifyBatch 500 on a fused plan); a final chains-only
    launch flushes the last cycle.  Every cycle a different request stream;
    request and batch digests bit-exact vs the oracle."""
    torch = _torch()
    stride = 16 + data_len
    idx, first = sharding.batch_lists(n, bs)
    plan = engine.pipeline(n, idx, first, np.full(n, stride), mode=mode)
    d_arena = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    d_off = torch.arange(n, dtype=torch.int64, device="cuda") * stride
    d_len = torch.full((n,), stride, dtype=torch.int32, device="cuda")
    d_req = [torch.empty((n, 32), dtype=torch.uint8, device="cuda") for _ in range(2)]
    d_bat = torch.empty((first.size - 1, 32), dtype=torch.uint8, device="cuda")
    want_req = []
    for i in range(cycles + 1):
        prev = d_req[(i + 1) % 2].data_ptr() if i else 0
        if i < cycles:
            seed = synth.SEED_BASE + 60 + i
            engine.synth_requests_device(seed, 0, n, data_len, d_arena.data_ptr())
            arena = oracle_py.gen_requests(seed, 0, n, data_len)
            want_req.append(oracle_py.hash_requests(arena, np.arange(n, dtype=np.uint64) * stride,
                                                    np.full(n, stride), threads=8))
            d_bat.zero_()
            torch.cuda.synchronize()
            engine.pipeline_overlap_device(plan, d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(),
                                           d_len.data_ptr(), d_req[i % 2].data_ptr(), prev, d_bat.data_ptr())
        else:  # flush: the last cycle's batches only
            d_bat.zero_()
            torch.cuda.synchronize()
            engine.pipeline_overlap_device(plan, 0, 0, 0, 0, 0, prev, d_bat.data_ptr())
        engine.sync()
        if i < cycles:
            assert np.array_equal(d_req[i % 2].cpu().numpy(), want_req[i]), f"cycle {i} requests"
        if i:
            assert np.array_equal(d_bat.cpu().numpy(), oracle_py.batch_digests(want_req[i - 1], idx, first)), \
                f"cycle {i - 1} batches"
    plan.close()


def test_pipeline_overlap_irregular_lists(engine):
    """Overlapped chains over compacted irregular lists (shared, unlisted and
    null entries, empty and odd lists) of a mixed-length request stream."""
    torch = _torch()
    arena, off, lens, idx, first = _irregular(51, 4000, 500, 70, 700)
    n = lens.size
    plan = engine.pipeline(n, idx, first, lens, mode="sequential")
    d_arena = torch.from_numpy(arena).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.from_numpy(lens.view(np.int32)).cuda()
    d_req = [torch.empty((n, 32), dtype=torch.uint8, device="cuda") for _ in range(2)]
    d_bat = torch.empty((first.size - 1, 32), dtype=torch.uint8, device="cuda")
    want_req = oracle_py.hash_requests(arena, off, lens)
    want_bat = oracle_py.batch_digests(want_req, idx, first)
    torch.cuda.synchronize()
    engine.pipeline_overlap_device(plan, d_arena.data_ptr(), arena.size, d_off.data_ptr(), d_len.data_ptr(),
                                   d_req[0].data_ptr(), 0, d_bat.data_ptr())
    engine.pipeline_overlap_device(plan, d_arena.data_ptr(), arena.size, d_off.data_ptr(), d_len.data_ptr(),
                                   d_req[1].data_ptr(), d_req[0].data_ptr(), d_bat.data_ptr())
    engine.sync()
    assert np.array_equal(d_req[0].cpu().numpy(), want_req)
    assert np.array_equal(d_req[1].cpu().numpy(), want_req)
    assert np.array_equal(d_bat.cpu().numpy(), want_bat)
    # the same two cycles on a fused plan (list pairs over the previous digests)
    fused = engine.pipeline(n, idx, first, lens, mode="fused")
    d_bat.zero_()
    torch.cuda.synchronize()
    engine.pipeline_overlap_device(fused, d_arena.data_ptr(), arena.size, d_off.data_ptr(), d_len.data_ptr(),
                                   d_req[0].data_ptr(), d_req[1].data_ptr(), d_bat.data_ptr())
    engine.sync()
    assert np.array_equal(d_req[0].cpu().numpy(), want_req)
    assert np.array_equal(d_bat.cpu().numpy(), want_bat)
    fused.status()
    # an ordinary fused run on the same plan afterwards (readiness epochs kept)
    for req, lst in _plan_run(engine, fused, arena, off, lens, first.size - 1, runs=1):
        assert np.array_equal(req, want_req)
        assert np.array_equal(lst, want_bat)
    fused.close()
    plan.close()


def _lists(kind, n, bs, rng):
    """(idx, first): identity BatchSize lists (the chain kernel's computed-index
    form) and near misses that must take the loaded-index form."""
    idx, first = sharding.batch_lists(n, bs)
    idx, first = idx.copy(), first.astype(np.int64)
    if kind == "permuted":  # uniform bounds, entries not the identity
        idx = rng.permutation(n).astype(np.uint32)
    elif kind == "short_middle" and first.size > 3:  # identity entries, one list cut short in the middle
        first = np.delete(first, 1)
        first = np.insert(first, 1, max(bs // 2, 1))
        first = np.maximum.accumulate(first)
    elif kind == "offset":  # identity lists not starting at request 0
        idx = idx[1:]
        first = np.minimum(first, idx.size)
    return idx.astype(np.uint32), first.astype(np.uint32)


@pytest.mark.parametrize("kind", ["identity", "permuted", "short_middle", "offset"])
# more than kPairMaxGroups x 64 = 32,768 lists: the chain kernel (fewer go to the pair kernel)
# even BatchSize: full lists end with a padding-only block (constant-schedule rounds)
@pytest.mark.parametrize("n,bs", [(40_000, 1), (70_001, 2), (80_000, 2), (245_763, 7), (700_003, 20),
                                  (655_380, 20)])
def test_pipeline_uniform_lists(engine, kind, n, bs):
    """Sequential plans over BatchSize lists: identity lists of one size run the
    chain kernel's computed-index form (round 6: no cfirst / cidx loads), every
    near miss the loaded-index form; both bit-exact vs the oracle, the final
    (short) list included."""
    rng = np.random.default_rng(n + bs)
    lens = rng.integers(0, 300, n).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(lens[:-1], out=off[1:])
    arena = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    idx, first = _lists(kind, n, bs, rng)
    plan = engine.pipeline(n, idx, first, lens, mode="sequential")
    assert plan.mode_name == "sequential"
    want_req = oracle_py.hash_requests(arena, off, lens)
    want_lst = oracle_py.batch_digests(want_req, idx, first)
    for req, lst in _plan_run(engine, plan, arena, off, lens, first.size - 1, runs=2):
        assert np.array_equal(req, want_req)
        assert np.array_equal(lst, want_lst)
    plan.close()


def _irregular(seed, n=3000, n_lists=300, max_list=60, max_len=600, min_len=0):
    rng = np.random.default_rng(seed)
    lens = rng.integers(min_len, max_len, n).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(lens[:-1], out=off[1:])
    arena = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    sizes = rng.integers(0, max_list, n_lists)
    sizes[::9] = 0
    idx = rng.integers(0, max(n // 2, 1), int(sizes.sum())).astype(np.uint32)  # half the requests unlisted
    idx[rng.random(idx.size) < 0.1] = _lib.MIRSHA_NULL_INDEX
    first = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    return arena, off, lens, idx, first


@pytest.mark.parametrize("env_mode", [None, "fused", "auto", "sequential"])
def test_pipeline_irregular_lists(engine, monkeypatch, env_mode):
    """Shared requests, unlisted requests, nulls, empty and odd lists through the
    host API (general path, or a per-call plan when MIRSHA_PIPELINE_MODE is set)."""
    if env_mode:
        monkeypatch.setenv("MIRSHA_PIPELINE_MODE", env_mode)
    arena, off, lens, idx, first = _irregular(21)
    req, bat = engine.hash_requests_then_batches(arena, off, lens, idx, first)
    want_req = oracle_py.hash_requests(arena, off, lens)
    assert np.array_equal(req, want_req)
    assert np.array_equal(bat, oracle_py.batch_digests(want_req, idx, first))


@pytest.mark.parametrize("seed,n,n_lists,max_list,max_len", [
    (31, 3000, 300, 60, 600),        # mixed lengths (bucketed order), shared / unlisted / null entries
    (32, 20000, 70000, 4, 300),      # list groups (1094) > half the grid's waves on small grids: role split
    (33, 64, 5, 1200, 100),          # few long chains over few tiles, heavy sharing
    (34, 1, 3, 40, 10),              # one request, repeated in every list
    (35, 5000, 2, 0, 2000),          # only empty lists (no entries): padding block only
])
@pytest.mark.parametrize("pace,list_tiles", [(1, 0), (2, 0), (4, 0), (1, 2), (3, 1), (4, 1), (4, 2)])
def test_fused_plan_irregular(engine, monkeypatch, pace, list_tiles, seed, n, n_lists, max_list, max_len):
    """Fused plan (device API) on irregular shapes, three runs on one plan (the
    tile queues' tickets carried across runs), 1-4 tile queues, list blocks
    with and without tile waves."""
    monkeypatch.setenv("MIRSHA_AB", "1")
    monkeypatch.setenv("MIRSHA_FUSED_PACE", str(pace))
    monkeypatch.setenv("MIRSHA_FUSED_LIST_TILES", str(list_tiles))
    arena, off, lens, idx, first = _irregular(seed, n, n_lists, max(max_list, 1), max_len)
    if max_list == 0:
        first = np.zeros(n_lists + 1, dtype=np.uint32)
        idx = np.zeros(0, dtype=np.uint32)
    plan = engine.pipeline(n, idx, first, lens, mode="fused")
    want_req = oracle_py.hash_requests(arena, off, lens)
    want_lst = oracle_py.batch_digests(want_req, idx, first)
    for req, lst in _plan_run(engine, plan, arena, off, lens, first.size - 1, runs=3):
        assert np.array_equal(req, want_req)
        assert np.array_equal(lst, want_lst)
    plan.close()


@pytest.mark.parametrize("list_tiles", [0, 1, 2])
def test_fused_list_tiles_config3(engine, monkeypatch, list_tiles):
    """Config 3 at full size (2^18 x 4 KB, VerifyBatch 500) on fused plans
    whose list blocks also run tile waves (MIRSHA_FUSED_LIST_TILES): two
    ordinary runs, then two overlapped cycles and the flush, bit-exact."""
    torch = _torch()
    monkeypatch.setenv("MIRSHA_AB", "1")
    monkeypatch.setenv("MIRSHA_FUSED_LIST_TILES", str(list_tiles))
    n, data_len, bs = 1 << 18, 4096, 500
    stride = 16 + data_len
    seed = synth.SEED_BASE + 3
    idx, first = sharding.batch_lists(n, bs)
    plan = engine.pipeline(n, idx, first, np.full(n, stride), mode="fused")
    d_arena = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    d_off = torch.arange(n, dtype=torch.int64, device="cuda") * stride
    d_len = torch.full((n,), stride, dtype=torch.int32, device="cuda")
    d_req = [torch.empty((n, 32), dtype=torch.uint8, device="cuda") for _ in range(2)]
    d_bat = torch.empty((first.size - 1, 32), dtype=torch.uint8, device="cuda")
    engine.synth_requests_device(seed, 0, n, data_len, d_arena.data_ptr())
    arena = oracle_py.gen_requests(seed, 0, n, data_len)
    want_req = oracle_py.hash_requests(arena, np.arange(n, dtype=np.uint64) * stride, np.full(n, stride), threads=8)
    want_bat = oracle_py.batch_digests(want_req, idx, first)
    args = (d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(), d_len.data_ptr())
    for _ in range(2):
        d_req[0].zero_()
        d_bat.zero_()
        torch.cuda.synchronize()  # torch's stream vs the engine's own (non-blocking) stream
        engine.hash_requests_then_batches_device(plan, *args, d_req[0].data_ptr(), d_bat.data_ptr())
        plan.status()
        assert np.array_equal(d_req[0].cpu().numpy(), want_req)
        assert np.array_equal(d_bat.cpu().numpy(), want_bat)
    for i in range(3):  # two cycles of the same stream, then the flush
        d_bat.zero_()
        prev = d_req[(i + 1) % 2].data_ptr() if i else 0
        if i < 2:
            d_req[i % 2].zero_()
        torch.cuda.synchronize()  # torch's stream vs the engine's own (non-blocking) stream
        if i < 2:
            engine.pipeline_overlap_device(plan, *args, d_req[i % 2].data_ptr(), prev, d_bat.data_ptr())
        else:
            engine.pipeline_overlap_device(plan, 0, 0, 0, 0, 0, prev, d_bat.data_ptr())
        engine.sync()
        if i < 2:
            assert np.array_equal(d_req[i % 2].cpu().numpy(), want_req), f"cycle {i} requests"
        if i:
            assert np.array_equal(d_bat.cpu().numpy(), want_bat), f"cycle {i - 1} batches"
    plan.status()
    plan.close()


@pytest.mark.parametrize("pace,n_tiles", [(1, 1100), (2, 2200), (4, 4200)])
def test_fused_split_tiles(engine, monkeypatch, pace, n_tiles):
    """More request tiles than the fused launch has tile-wave slots: the
    overflow tiles run as block-range segments (midstate through memory,
    sequential flags) interleaved in the last queue's tiles.  Mixed
    lengths (split tiles of different block counts than their hosts'), shared
    / null list entries; three runs on one plan (monotone segment flags), then
    overlapped cycles and the flush; bit-exact vs the oracle."""
    torch = _torch()
    monkeypatch.setenv("MIRSHA_AB", "1")
    monkeypatch.setenv("MIRSHA_FUSED_PACE", str(pace))
    arena, off, lens, idx, first = _irregular(60 + pace, 64 * n_tiles - 17, 2048, 60, 1300, 300)
    plan = engine.pipeline(lens.size, idx, first, lens, mode="fused")
    n_split, per_tile = plan.split_tiles()
    assert n_split > 0 and per_tile >= 2, (n_split, per_tile)
    want_req = oracle_py.hash_requests(arena, off, lens, threads=8)
    want_lst = oracle_py.batch_digests(want_req, idx, first)
    for req, lst in _plan_run(engine, plan, arena, off, lens, first.size - 1, runs=3):
        assert np.array_equal(req, want_req)
        assert np.array_equal(lst, want_lst)
    d_arena = torch.from_numpy(arena).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.from_numpy(lens.view(np.int32)).cuda()
    d_req = [torch.zeros((lens.size, 32), dtype=torch.uint8, device="cuda") for _ in range(2)]
    d_lst = torch.zeros((first.size - 1, 32), dtype=torch.uint8, device="cuda")
    args = (d_arena.data_ptr(), arena.size, d_off.data_ptr(), d_len.data_ptr())
    torch.cuda.synchronize()
    engine.pipeline_overlap_device(plan, *args, d_req[0].data_ptr(), 0, d_lst.data_ptr())
    engine.pipeline_overlap_device(plan, *args, d_req[1].data_ptr(), d_req[0].data_ptr(), d_lst.data_ptr())
    engine.sync()
    plan.status()
    assert np.array_equal(d_req[0].cpu().numpy(), want_req)
    assert np.array_equal(d_req[1].cpu().numpy(), want_req)
    assert np.array_equal(d_lst.cpu().numpy(), want_lst)
    plan.close()


def test_fused_split_tiles_shorter_run_lengths(engine, monkeypatch):
    """A plan's split-tile segment ranges are cut from the lengths given at
    plan creation (a bucketing hint); runs may pass other lengths.  Here the
    run-time messages are prefixes of the planned ones (a third to a half of
    their blocks), so a middle segment finishes each split tile and the later
    segments must do nothing: no second digest store, no second readiness
    increment.  Runs with the short lengths, then the planned
    lengths, then the short ones again on one plan; bit-exact every time."""
    monkeypatch.setenv("MIRSHA_AB", "1")
    monkeypatch.setenv("MIRSHA_FUSED_PACE", "2")
    arena, off, lens, idx, first = _irregular(77, 64 * 2200 - 5, 1024, 60, 1300, 900)
    plan = engine.pipeline(lens.size, idx, first, lens, mode="fused")
    n_split, per_tile = plan.split_tiles()
    assert n_split > 0 and per_tile >= 2, (n_split, per_tile)
    short = (lens // 3).astype(np.uint32)
    for run_lens in (short, lens, short):
        want_req = oracle_py.hash_requests(arena, off, run_lens, threads=8)
        want_lst = oracle_py.batch_digests(want_req, idx, first)
        for req, lst in _plan_run(engine, plan, arena, off, run_lens, first.size - 1, runs=2):
            assert np.array_equal(req, want_req)
            assert np.array_equal(lst, want_lst)
    plan.close()


@pytest.mark.parametrize("placement", ["broken", "remap"])
def test_fused_placement_fallback(engine, monkeypatch, placement):
    """The fused launch deals its static roles (first tiles, list pair,
    segment hosts) by (SIMD, slot).  broken: the plan's placement probe is
    made to report a non-cyclic dealing (test knob), and the fused plan is
    built sequential instead (mirsha_pipeline_fallback = 1); remap: the plan
    stays fused but every wave of the launch reads SIMD 0, so the kernel's
    identity remap hands the missing (SIMD, slot) roles to the extra waves.
    Both bit-exact at config-3 shape on a reduced count (split tiles
    included), over two runs and an overlapped cycle."""
    torch = _torch()
    monkeypatch.setenv("MIRSHA_AB", "1")
    monkeypatch.setenv("MIRSHA_TEST_PLACEMENT", placement)
    n, data_len, bs = 64 * 4100, 4096, 500
    stride = 16 + data_len
    seed = synth.SEED_BASE + 80
    idx, first = sharding.batch_lists(n, bs)
    plan = engine.pipeline(n, idx, first, np.full(n, stride), mode="fused")
    monkeypatch.delenv("MIRSHA_TEST_PLACEMENT")
    if placement == "broken":
        assert plan.mode_name == "sequential" and plan.fallback == 1
    else:
        assert plan.mode_name == "fused" and plan.fallback == 0
        assert plan.split_tiles()[0] > 0
    d_arena = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    d_off = torch.arange(n, dtype=torch.int64, device="cuda") * stride
    d_len = torch.full((n,), stride, dtype=torch.int32, device="cuda")
    d_req = [torch.empty((n, 32), dtype=torch.uint8, device="cuda") for _ in range(2)]
    d_bat = torch.empty((first.size - 1, 32), dtype=torch.uint8, device="cuda")
    engine.synth_requests_device(seed, 0, n, data_len, d_arena.data_ptr())
    arena = oracle_py.gen_requests(seed, 0, n, data_len)
    want_req = oracle_py.hash_requests(arena, np.arange(n, dtype=np.uint64) * stride, np.full(n, stride), threads=8)
    want_bat = oracle_py.batch_digests(want_req, idx, first)
    args = (d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(), d_len.data_ptr())
    for _ in range(2):
        d_req[0].zero_()
        d_bat.zero_()
        torch.cuda.synchronize()
        engine.hash_requests_then_batches_device(plan, *args, d_req[0].data_ptr(), d_bat.data_ptr())
        plan.status()
        assert np.array_equal(d_req[0].cpu().numpy(), want_req)
        assert np.array_equal(d_bat.cpu().numpy(), want_bat)
    d_bat.zero_()
    d_req[1].zero_()
    torch.cuda.synchronize()
    engine.pipeline_overlap_device(plan, *args, d_req[1].data_ptr(), d_req[0].data_ptr(), d_bat.data_ptr())
    engine.sync()
    plan.status()
    assert np.array_equal(d_req[1].cpu().numpy(), want_req)
    assert np.array_equal(d_bat.cpu().numpy(), want_bat)
    plan.close()


@pytest.mark.parametrize("lone,deep", [("1", "1"), ("0", "1"), ("1", "0"), ("0", "0")])
def test_fused_lone_stretch_forms(engine, monkeypatch, lone, deep):
    """The last queue's lone stretch (hash_tile in the fused launch): the
    latency round form once the wave is alone on its SIMD (g_simd_live) and
    the two-blocks-ahead staging, each on and off (MIRSHA_FUSED_LONE_FORM,
    MIRSHA_FUSED_DEEP_LAST): config-3-shaped tiles plus split tiles, three
    runs and an overlapped cycle, bit-exact vs the oracle every way."""
    torch = _torch()
    monkeypatch.setenv("MIRSHA_AB", "1")
    monkeypatch.setenv("MIRSHA_FUSED_LONE_FORM", lone)
    monkeypatch.setenv("MIRSHA_FUSED_DEEP_LAST", deep)
    n, stride = 64 * 4100 - 3, 16 + 4096
    seed = synth.SEED_BASE + 90
    arena = oracle_py.gen_requests(seed, 0, n, 4096)
    off = np.arange(n, dtype=np.uint64) * stride
    lens = np.full(n, stride, dtype=np.uint32)
    idx, first = sharding.batch_lists(n, 500)
    plan = engine.pipeline(n, idx, first, lens, mode="fused")
    assert plan.mode_name == "fused" and plan.split_tiles()[0] > 0
    want_req = oracle_py.hash_requests(arena, off, lens, threads=8)
    want_lst = oracle_py.batch_digests(want_req, idx, first)
    for req, lst in _plan_run(engine, plan, arena, off, lens, first.size - 1, runs=3):
        assert np.array_equal(req, want_req)
        assert np.array_equal(lst, want_lst)
    d_arena = torch.from_numpy(arena).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.from_numpy(lens.view(np.int32)).cuda()
    d_req = [torch.zeros((n, 32), dtype=torch.uint8, device="cuda") for _ in range(2)]
    d_lst = torch.zeros((first.size - 1, 32), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    args = (d_arena.data_ptr(), arena.size, d_off.data_ptr(), d_len.data_ptr())
    engine.pipeline_overlap_device(plan, *args, d_req[0].data_ptr(), 0, d_lst.data_ptr())
    engine.pipeline_overlap_device(plan, *args, d_req[1].data_ptr(), d_req[0].data_ptr(), d_lst.data_ptr())
    engine.sync()
    plan.status()
    assert np.array_equal(d_req[1].cpu().numpy(), want_req)
    assert np.array_equal(d_lst.cpu().numpy(), want_lst)
    plan.close()


def test_fused_watchdog_fails_closed(engine, monkeypatch):
    """A fused run whose readiness waits expire (test-only zero watchdog,
    MIRSHA_TEST_FUSED_WATCHDOG=0) fails closed: the plan's status is
    MIRSHA_EHIP, no list digest is written (the output keeps its fill byte),
    and every later run on the plan is refused without a synchronisation.
    Request digests are unaffected (tiles never wait).  A new plan with the
    default watchdog is bit-exact again."""
    torch = _torch()
    n, data_len, bs = 20_000, 4096, 500
    stride = 16 + data_len
    seed = synth.SEED_BASE + 70
    idx, first = sharding.batch_lists(n, bs)
    d_arena = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    d_off = torch.arange(n, dtype=torch.int64, device="cuda") * stride
    d_len = torch.full((n,), stride, dtype=torch.int32, device="cuda")
    d_req = torch.zeros((n, 32), dtype=torch.uint8, device="cuda")
    d_bat = torch.full((first.size - 1, 32), 0xA5, dtype=torch.uint8, device="cuda")
    engine.synth_requests_device(seed, 0, n, data_len, d_arena.data_ptr())
    want_req = oracle_py.hash_requests(oracle_py.gen_requests(seed, 0, n, data_len),
                                       np.arange(n, dtype=np.uint64) * stride, np.full(n, stride), threads=8)
    args = (d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(), d_len.data_ptr())
    monkeypatch.setenv("MIRSHA_AB", "1")
    monkeypatch.setenv("MIRSHA_TEST_FUSED_WATCHDOG", "0")
    plan = engine.pipeline(n, idx, first, np.full(n, stride), mode="fused")
    monkeypatch.delenv("MIRSHA_TEST_FUSED_WATCHDOG")
    torch.cuda.synchronize()
    engine.hash_requests_then_batches_device(plan, *args, d_req.data_ptr(), d_bat.data_ptr())
    with pytest.raises(MirshaError) as e:
        plan.status()
    assert e.value.code == _lib.MIRSHA_EHIP
    assert (d_bat.cpu().numpy() == 0xA5).all(), "a list digest was stored after the watchdog expired"
    assert np.array_equal(d_req.cpu().numpy(), want_req)
    with pytest.raises(MirshaError) as e:
        engine.hash_requests_then_batches_device(plan, *args, d_req.data_ptr(), d_bat.data_ptr())
    assert e.value.code == _lib.MIRSHA_EHIP
    with pytest.raises(MirshaError) as e:
        engine.pipeline_overlap_device(plan, *args, d_req.data_ptr(), d_req.data_ptr(), d_bat.data_ptr())
    assert e.value.code == _lib.MIRSHA_EHIP
    plan.close()
    fresh = engine.pipeline(n, idx, first, np.full(n, stride), mode="fused")
    torch.cuda.synchronize()
    engine.hash_requests_then_batches_device(fresh, *args, d_req.data_ptr(), d_bat.data_ptr())
    fresh.status()
    assert np.array_equal(d_bat.cpu().numpy(), oracle_py.batch_digests(want_req, idx, first))
    fresh.close()


def test_fused_plans_interleaved(engine, monkeypatch):
    """Two fused plans used alternately: each keeps its own tickets / counters
    (3 and 4 tile queues)."""
    a = _irregular(41, 2000, 200, 40, 400)
    b = _irregular(42, 5000, 90, 300, 200)
    monkeypatch.setenv("MIRSHA_AB", "1")
    monkeypatch.setenv("MIRSHA_FUSED_PACE", "3")
    pa = engine.pipeline(a[2].size, a[3], a[4], a[2], mode="fused")
    monkeypatch.setenv("MIRSHA_FUSED_PACE", "4")
    pb = engine.pipeline(b[2].size, b[3], b[4], b[2], mode="fused")
    for _ in range(2):
        for (arena, off, lens, idx, first), plan in ((a, pa), (b, pb)):
            want_req = oracle_py.hash_requests(arena, off, lens)
            (req, lst), = _plan_run(engine, plan, arena, off, lens, first.size - 1, runs=1)
            assert np.array_equal(req, want_req)
            assert np.array_equal(lst, oracle_py.batch_digests(want_req, idx, first))
    pa.close()
    pb.close()


def test_config5_generator_and_wide_arena(engine):
    """Config-5 mixed-size generator (device) vs the oracle, and the 64-bit
    addressed loader on an arena > 4 GiB: messages packed at the start, past
    4 GiB, and ending exactly at arena_len (range-checked tail)."""
    torch = _torch()
    seed, first, n = synth.SEED_BASE + 5, 10**7 + 3, 1500
    d_len = torch.empty(n, dtype=torch.int32, device="cuda")
    engine.synth_mixed_lengths_device(seed, first, n, d_len.data_ptr())
    engine.sync()
    ln = d_len.cpu().numpy().view(np.uint32)
    arena_o, off_o, ln_o = oracle_py.gen_mixed(seed, np.arange(first, first + n, dtype=np.uint64))
    assert np.array_equal(ln, ln_o)
    # first half packed from 0 (odd start), second half packed to end exactly at arena_len > 4 GiB
    half = n // 2
    off = np.zeros(n, dtype=np.uint64)
    off[:half] = 3 + np.concatenate([[0], np.cumsum(ln[:half - 1], dtype=np.uint64)])
    tail = int(ln[half:].sum())
    arena_len = (1 << 32) + 12345 + tail
    off[half:] = arena_len - tail + np.concatenate([[0], np.cumsum(ln[half:-1], dtype=np.uint64)])
    d_arena = torch.zeros(arena_len, dtype=torch.uint8, device="cuda")
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    engine.synth_mixed_device(seed, first, n, d_off.data_ptr(), d_arena.data_ptr())
    engine.sync()
    # bytes of a few messages vs the oracle
    for k in (0, 1, half - 1, half, n - 1):
        got = d_arena[int(off[k]):int(off[k]) + int(ln[k])].cpu().numpy()
        want = arena_o[int(off_o[k]):int(off_o[k]) + int(ln_o[k])]
        assert np.array_equal(got, want), k
    want = oracle_py.hash_requests(arena_o, off_o, ln_o)
    from mirbft_amd import bucket_order

    order, _ = bucket_order(ln)
    d_out = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    for d_order in (None, torch.from_numpy(order.view(np.int32)).cuda()):
        d_out.zero_()
        torch.cuda.synchronize()  # torch's stream vs the engine's own (non-blocking) stream
        engine.hash_batch_device(d_arena.data_ptr(), arena_len, d_off.data_ptr(), d_len.data_ptr(),
                                 None if d_order is None else d_order.data_ptr(), n, d_out.data_ptr())
        engine.sync()
        assert np.array_equal(d_out.cpu().numpy(), want)


def _contiguous(seed, n, bs, listed, max_len):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, max_len, n).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(lens[:-1], out=off[1:])
    arena = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    idx, first = sharding.batch_lists(listed, bs)
    return arena, off, lens, idx, first


@pytest.mark.parametrize("variant", [11, 12, 13, 14, 15])
def test_ab_forms_not_in_product_library(engine, variant, monkeypatch):
    """Variants 11-15 (retired and diagnostic CU-block forms; 14 skips its
    loads and writes wrong digests) live only in the tools A/B build: the
    product library refuses them even with MIRSHA_AB=1."""
    if os.environ.get("MIRSHA_AB_LIB"):
        pytest.skip("an A/B build is loaded")
    monkeypatch.setenv("MIRSHA_AB", "1")
    with pytest.raises(MirshaError) as e:
        engine.set_variant(variant)
    assert e.value.code == _lib.MIRSHA_EINVAL
    assert _hex(engine.hash_messages([b"abc"])) == [
        "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"]


@pytest.mark.parametrize("variant", [2, 3, 7, 8, 9, -1])
def test_retired_variants_rejected(engine, variant):
    """Round-1 A/B kernel forms are out of the product: EINVAL, not a silent default."""
    with pytest.raises(MirshaError) as e:
        engine.set_variant(variant)
    assert e.value.code == _lib.MIRSHA_EINVAL


@pytest.mark.parametrize("mode", [2, 4, 5])
def test_retired_pipeline_modes_rejected(engine, mode):
    idx, first = sharding.batch_lists(64, 20)
    with pytest.raises(MirshaError) as e:
        engine.pipeline(64, idx, first, np.full(64, 272), mode=mode)
    assert e.value.code == _lib.MIRSHA_EINVAL


def test_clock_probe_sane(engine):
    """The bench's clock probe: a clock within the part's range and a
    compression cost no cheaper than the spec issue floor (2 x 1,384 cycles)."""
    ghz, cyc = engine.clock_probe(8)
    assert 0.5 < ghz < 3.0
    assert 2 * 1384 <= cyc < 50000
