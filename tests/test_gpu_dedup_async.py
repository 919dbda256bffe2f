"""GPU parity of the dedup and asynchronous, order-preserving
(§8 f3) entry points, through the C-ABI: bit-exact against hashlib (the
FIPS 180-4 oracle, pinned in test_oracle_golden.py) in origin order."""
import ctypes
import hashlib

import numpy as np
import pytest

from mirbft_amd import (Actions, HashRequest, Processor, ProcessorWorkPool, SliceArrays, hashdata)
from mirbft_amd import _lib
from test_host_dedup import python_plan, random_requests

pytestmark = pytest.mark.gpu


def want(requests):
    return [hashlib.sha256(b"".join(bytes(s) for s in r)).digest() for r in requests]


def rows(a):
    return [r.tobytes() for r in a]


@pytest.mark.parametrize("seed", [0, 1])
def test_dedup_random(engine, seed):
    reqs = random_requests(seed, n=500)
    got = engine.hash_slices(reqs, dedup=True)
    assert rows(got) == want(reqs)
    assert engine.last_unique == python_plan(reqs)[1]


def test_dedup_epoch_change_cycle(engine):
    n_nodes, n_req = 16, 256  # every origin relayed by 16 sources
    buf, so, sl, first, origin = hashdata.epoch_change_cycle(n_nodes, n_req, 3, 120, 120)
    arrays = SliceArrays.from_buffer(buf, so, sl, first)
    got = engine.hash_slice_arrays(arrays, dedup=True)
    assert engine.last_unique == n_nodes
    payload = [hashlib.sha256(hashdata.concat(hashdata.epoch_change_payload(2, o, 3, 120, 120))).digest()
               for o in range(n_nodes)]
    assert rows(got) == [payload[o] for o in origin]
    plain = engine.hash_slice_arrays(arrays, dedup=False)
    assert np.array_equal(plain, got)


def test_dedup_all_distinct_and_all_equal(engine):
    distinct = [[bytes([i]) * (i + 1)] for i in range(100)]
    assert rows(engine.hash_slices(distinct, dedup=True)) == want(distinct)
    assert engine.last_unique == 100
    same = [[b"x" * 5000]] * 77 + [[b"x" * 2500, b"x" * 2500]]
    assert rows(engine.hash_slices(same, dedup=True)) == want(same)
    assert engine.last_unique == 1
    empties = [[], [b""], [b"", b""]]
    assert rows(engine.hash_slices(empties, dedup=True)) == want(empties)
    assert engine.last_unique == 1
    assert engine.hash_slices([], dedup=True).shape == (0, 32)


def test_async_order_and_ring_retirement(engine):
    """Nine submissions (more than the 4-slot ring) of different shapes, some
    deduplicated; waits out of order; every ticket's digests in origin order."""
    batches = [random_requests(s, n=50 + 40 * s) for s in range(9)]
    tickets = [engine.submit_slices(b, dedup=bool(s % 2)) for s, b in enumerate(batches)]
    assert [t.value for t in tickets] == sorted(t.value for t in tickets)
    # waiting for a later ticket completes every earlier one too
    assert rows(engine.wait(tickets[5])) == want(batches[5])
    for s in (0, 3, 1, 2, 4):
        assert engine.poll(tickets[s])
        assert rows(tickets[s].out) == want(batches[s])
    for s in (8, 6, 7):
        assert rows(engine.wait(tickets[s])) == want(batches[s])


def test_async_poll_and_empty_submission(engine):
    t0 = engine.submit_slices([])
    assert engine.wait(t0).shape == (0, 32)
    reqs = [[b"abc"] * k for k in range(1, 200)]
    t = engine.submit_slices(reqs)
    while not engine.poll(t):
        pass
    assert rows(t.out) == want(reqs)


def test_async_caller_may_reuse_slices_after_submit(engine):
    buf = bytearray(b"q" * 4096)
    arr = np.frombuffer(buf, dtype=np.uint8)
    sl = SliceArrays.from_buffer(arr, np.arange(64, dtype=np.uint64) * 64, np.full(64, 64, dtype=np.uint64),
                                 np.arange(65, dtype=np.uint32))
    t = engine.submit_slices(sl)
    expect = [hashlib.sha256(bytes(buf[64 * i: 64 * i + 64])).digest() for i in range(64)]
    arr[:] = 0  # the library packed the bytes before submit returned
    assert rows(engine.wait(t)) == expect


def test_invalid_ticket_raises(engine):
    from mirbft_amd import MirshaError
    from mirbft_amd.engine import Ticket

    with pytest.raises(MirshaError):
        engine.wait(Ticket(10 ** 9, np.empty((0, 32), np.uint8)))
    sl = SliceArrays.from_requests([[b"a"]])
    out = np.empty((1, 32), np.uint8)
    t = ctypes.c_uint64(0)
    with pytest.raises(MirshaError):  # unknown flag bit
        engine._check(engine._lib.mirsha_submit_slices(engine.ctx, sl.ptr_p, sl.len_p, sl.first_p, 1,
                                                       out.ctypes.data, 0x80, ctypes.byref(t)))


def test_processor_dedup_and_submit(engine):
    reqs = [HashRequest(data=d, origin=i) for i, d in enumerate(random_requests(7, n=120))]
    p = Processor(engine, dedup=True)
    r = p.process(Actions(hash=reqs))
    assert [x.request for x in r.digests] == reqs
    assert [x.digest for x in r.digests] == want([q.data for q in reqs])
    pending = Processor(engine).submit(Actions(hash=reqs))
    r2 = pending.wait()
    assert [x.request for x in r2.digests] == reqs
    assert [x.digest for x in r2.digests] == want([q.data for q in reqs])
    assert pending.done()
    assert Processor(engine).submit(Actions(hash=[])).wait().digests == []


def test_work_pool_overlap(engine):
    reqs = [HashRequest(data=d) for d in random_requests(8, n=90)]
    ran = []
    r = ProcessorWorkPool(engine, dedup=True).process(Actions(hash=reqs), overlap=lambda: ran.append(1))
    assert ran == [1]
    assert [x.digest for x in r.digests] == want([q.data for q in reqs])
    assert [x.request for x in r.digests] == reqs


@pytest.mark.parametrize("flags", [1, 2, 3, 4, 5])
def test_cpp_mirror_dedup_async(flags):
    host = ctypes.CDLL(_lib.HOST_LIB_PATH)
    msgs = [b"m" * (i % 7) * 50 for i in range(100)]
    bufs = [ctypes.create_string_buffer(m, len(m) or 1) for m in msgs]
    data = (ctypes.c_void_p * len(msgs))(*[ctypes.addressof(b) for b in bufs])
    lens = (ctypes.c_uint64 * len(msgs))(*[len(m) for m in msgs])
    out = (ctypes.c_uint8 * (32 * len(msgs)))()
    uniq = ctypes.c_uint32(0)
    err = ctypes.create_string_buffer(256)
    host.mirbft_host_process_ex.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p,
                                            ctypes.c_uint32]
    rc = host.mirbft_host_process_ex(0, data, lens, len(msgs), out, flags, ctypes.byref(uniq), err, 256)
    assert rc == 0, err.value
    got = [bytes(out[32 * i: 32 * i + 32]) for i in range(len(msgs))]
    assert got == [hashlib.sha256(m).digest() for m in msgs]
    assert uniq.value == (7 if flags & 1 else len(msgs))


def test_config4_full_scale_epoch_change_cycle(engine):
    """BASELINE config 4 at its stated scale: a 64-node network's epoch change
    (mirbft.go:125-154: CheckpointInterval 320), one node's Ready() cycle =
    64 origins x 64 relaying sources of EpochChangeAck hash requests
    (applyEpochChangeAckMsg, epoch_target.go:459-477), each the
    epochChangeHashData slices of its origin's EpochChange
    (stateless.go:311-340): C = 3 checkpoints, |P| = |Q| = 640 entries,
    61,568-byte payloads of 3,847 slices, every ack its own copy (252 MB).
    Every digest, in origin order, equals hashlib over that origin's payload,
    through the dedup entry point, the plain one and the async submit."""
    n_nodes, n_req, cps, np_, nq = 64, 4096, 3, 640, 640
    buf, so, sl, first, origin = hashdata.epoch_change_cycle(n_nodes, n_req, cps, np_, nq)
    plen = buf.size // n_req
    assert plen == 8 + cps * 40 + (np_ + nq) * 48 == 61_568
    assert int(first[1]) == 1 + 2 * cps + 3 * (np_ + nq) == 3_847
    arrays = SliceArrays.from_buffer(buf, so, sl, first)
    payload = [hashlib.sha256(hashdata.concat(hashdata.epoch_change_payload(2, o, cps, np_, nq))).digest()
               for o in range(n_nodes)]
    expect = [payload[o] for o in origin]
    # the bytes of every ack are the origin's payload (not only equal digests)
    for r in (0, 1, 63, 64, 4095):
        assert hashlib.sha256(buf[r * plen:(r + 1) * plen].tobytes()).digest() == payload[origin[r]]
    got = engine.hash_slice_arrays(arrays, dedup=True)
    assert engine.last_unique == n_nodes
    assert rows(got) == expect
    prof = engine.host_profile()
    assert prof["plan"] > 0 and prof["device"] > 0
    plain = engine.hash_slice_arrays(arrays, dedup=False)
    assert engine.last_unique == n_req
    assert rows(plain) == expect
    t = engine.submit_slices(arrays, dedup=True)
    assert rows(engine.wait(t)) == expect


def test_dropped_ticket_then_four_more(engine):
    """a ticket dropped without wait() is retired by a later submit
    writing its digests; the engine keeps that output alive until then."""
    import gc

    reqs = [random_requests(s, n=64) for s in range(6)]
    t0 = engine.submit_slices(reqs[0])
    del t0
    gc.collect()
    ts = [engine.submit_slices(r) for r in reqs[1:5]]  # the 5th submission overall retires the dropped one
    assert len(engine._outstanding) <= 4
    for t, r in zip(ts, reqs[1:5]):
        assert rows(engine.wait(t)) == want(r)
    assert not engine._outstanding


@pytest.mark.parametrize("knobs", [{"MIRSHA_DEDUP_WEAK_FP": "1"},
                                   {"MIRSHA_DEDUP_SEGMENT_SLICES": "40"},
                                   {"MIRSHA_DEDUP_WEAK_FP": "1", "MIRSHA_DEDUP_SEGMENT_SLICES": "40"}])
def test_dedup_collision_path_second_launch(knobs):
    """Test hooks read once per process, hence a subprocess.
    MIRSHA_DEDUP_WEAK_FP=1: every fingerprint is equal, so the heads queued
    before the byte-for-byte confirmation are only one request per length, and
    every other distinct request is found by the confirmation and hashed in
    the second launch.  MIRSHA_DEDUP_SEGMENT_SLICES=40: the streamed scan in
    segments of ~40 slices, the first segment's heads launched before the rest
    is scanned, later heads in the second launch; a malformed request in a
    later segment (after the first launch was queued) fails the call and the
    context hashes on.  Digests in origin order, dedup count exact, sync and
    async forms."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import sys, hashlib; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
        "import torch; torch.cuda.is_available()\n"
        "import test_host_dedup as t\n"
        "from mirbft_amd import Engine\n"
        "e = Engine(0)\n"
        "for seed in (0, 1, 2):\n"
        "    reqs = t.random_requests(seed, n=300)\n"
        "    want = [hashlib.sha256(b''.join(bytes(s) for s in r)).digest() for r in reqs]\n"
        "    got = e.hash_slices(reqs, dedup=True)\n"
        "    assert [r.tobytes() for r in got] == want, seed\n"
        "    assert e.last_unique == t.python_plan(reqs)[1], seed\n"
        "    tk = e.submit_slices(reqs, dedup=True)\n"
        "    assert [r.tobytes() for r in e.wait(tk)] == want, seed\n"
        "from mirbft_amd import SliceArrays\n"
        "from mirbft_amd._lib import MirshaError\n"
        "sl = SliceArrays.from_requests([[bytes([i & 7]) * 70, b'c'] for i in range(60)])\n"
        "sl.ptr[101] = 0\n"
        "try:\n"
        "    e.hash_slice_arrays(sl, dedup=True)\n"
        "    raise SystemExit('no error')\n"
        "except MirshaError as x:\n"
        "    assert 'request 50' in str(x), str(x)\n"
        "ok = [[b'abc', b'def'], [b'abcdef'], [b'xyz']]\n"
        "assert [r.tobytes() for r in e.hash_slices(ok, dedup=True)] == [hashlib.sha256(b''.join(r)).digest() for r in ok]\n"
        "e.close()\n"
        "print('ok')\n" % (root, os.path.join(root, "tests"))
    )
    env = dict(os.environ, MIRSHA_AB="1", **knobs)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


@pytest.mark.parametrize("case", ["null_slice", "not_monotone", "too_long"])
def test_slice_argument_errors_dedup_and_plain(engine, case):
    """Invalid slice arrays are rejected the same way by the dedup call (whose
    validation rides in its fingerprint walk) and the plain one: same code,
    same first offending request, no byte read past a too-long request's
    limit (its slice is a 16-byte buffer declared 4 GiB long), and the
    context still hashes afterwards."""
    from mirbft_amd import SliceArrays
    from mirbft_amd._lib import MirshaError

    keep = [np.frombuffer(bytes(range(16)), dtype=np.uint8).copy() for _ in range(6)]
    ptr = np.array([k.ctypes.data for k in keep], dtype=np.uint64)
    ln = np.full(6, 16, dtype=np.uint64)
    first = np.array([0, 2, 4, 6], dtype=np.uint32)
    want_code, bad = _lib.MIRSHA_EINVAL, 1
    if case == "null_slice":
        ptr[3] = 0
    elif case == "not_monotone":
        first = np.array([0, 4, 2, 6], dtype=np.uint32)
    else:
        ln[3] = 1 << 32
        want_code = _lib.MIRSHA_ERANGE
    sl = SliceArrays(ptr, ln, first, keep)
    for dedup in (True, False):
        with pytest.raises(MirshaError) as e:
            engine.hash_slice_arrays(sl, dedup=dedup)
        assert e.value.code == want_code
        assert f"request {bad}" in str(e.value), str(e.value)
    ok = [[b"abc", b"def"], [b"abcdef"], [b"xyz"]]
    assert rows(engine.hash_slices(ok, dedup=True)) == want(ok)
