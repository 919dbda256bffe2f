"""Event-log writer/reader (eventlog/interceptor.go:301-378),
following the reference's own tests (eventlog/interceptor_test.go:29-105):
the two-tick log is 46 bytes, reads back event by event then EOF, and a
truncated stream fails with the reference's message.  The GPU test re-hashes
the payload-carrying hash results of a retained log through the engine."""
import gzip
import hashlib
import io
import random

import pytest

from mirbft_amd import eventlog as el
from mirbft_amd import hashdata

TICK = el.tick_event()


def two_tick_log(**kw):
    out = io.BytesIO()
    rec = el.Recorder(1, out, time_source=lambda: 2, **kw)
    rec.intercept(TICK)
    rec.intercept(TICK)
    rec.stop()
    return out.getvalue()


def test_recorder_two_ticks_is_46_bytes():
    # interceptor_test.go:38-50 (BufferSizeOpt(3): no effect on the bytes)
    data = two_tick_log(buffer_size=3)
    assert len(data) == 46
    # Go gzip header at BestSpeed: mtime 0, XFL 4, OS 255
    assert data[:10] == bytes.fromhex("1f8b08000000000004ff")
    rec = bytes.fromhex("10" "0801" "1002" "1a02" "4a00")  # zig-zag varint 8, RecordedEvent{1, 2, Tick}
    assert gzip.decompress(data) == rec + rec


def test_reader_round_trip_then_eof():
    # interceptor_test.go:74-94
    r = el.Reader(io.BytesIO(two_tick_log()))
    want = el.RecordedEvent(node_id=1, time=2, state_event=TICK)
    assert r.read_event() == want
    assert r.read_event() == want
    with pytest.raises(EOFError):
        r.read_event()


def test_truncated_stream_error():
    # interceptor_test.go:96-104
    data = two_tick_log()[:2]
    with pytest.raises(el.EventLogError, match="^could not read source as a gzip stream: unexpected EOF$"):
        el.Reader(io.BytesIO(data))
    with pytest.raises(el.EventLogError, match="^could not read source as a gzip stream: EOF$"):
        el.Reader(io.BytesIO(b""))


def test_truncated_body_errors():
    data = two_tick_log()
    r = el.Reader(io.BytesIO(data[:-8]))  # no gzip trailer
    r.read_event()
    r.read_event()
    with pytest.raises(el.EventLogError, match="unexpected EOF"):
        r.read_event()


@pytest.mark.parametrize("v,enc", [(0, "00"), (-1, "01"), (1, "02"), (63, "7e"), (-64, "7f"), (64, "8001"),
                                   (8, "10"), (-(1 << 63), "ffffffffffffffffff01"), ((1 << 63) - 1, "feffffffffffffffff01")])
def test_varint_matches_encoding_binary(v, enc):
    # binary.PutVarint / ReadVarint (interceptor.go:312, :359)
    assert el.put_varint(v).hex() == enc
    b = io.BytesIO(bytes.fromhex(enc))
    assert el.read_varint(lambda: (lambda c: c[0] if c else None)(b.read(1))) == v


def test_varint_cut_and_overflow():
    src = iter([0x80])
    with pytest.raises(el.EventLogError, match="unexpected EOF"):
        el.read_varint(lambda: next(src, None))
    src = iter([0xFF] * 10 + [0x01])
    with pytest.raises(el.EventLogError, match="overflows"):
        el.read_varint(lambda: next(src, None))


def request_msg(cid, rno, data):
    return el.f_uint(1, cid) + el.f_uint(2, rno) + el.f_bytes(3, data)


def ack_msg(cid, rno, digest):
    return el.f_uint(1, cid) + el.f_uint(2, rno) + el.f_bytes(3, digest)


def add_results(results, checkpoints=()):
    body = b"".join(el.f_msg(1, r) for r in results) + b"".join(el.f_msg(2, c) for c in checkpoints)
    return el.f_msg(el.SE_ADD_RESULTS, body)


def request_result(src, cid, rno, data):
    d = hashlib.sha256(hashdata.concat(hashdata.request_hash_data(cid, rno, data))).digest()
    return el.f_bytes(1, d) + el.f_msg(el.HR_REQUEST, el.f_uint(1, src) + el.f_msg(2, request_msg(cid, rno, data)))


def verify_result(src, cid, rno, data):
    d = hashlib.sha256(hashdata.concat(hashdata.request_hash_data(cid, rno, data))).digest()
    body = el.f_uint(1, src) + el.f_msg(2, ack_msg(cid, rno, d)) + el.f_bytes(3, data)
    return el.f_bytes(1, d) + el.f_msg(el.HR_VERIFY_REQUEST, body)


def batch_result(src, seq, digests):
    acks = b"".join(el.f_msg(5, ack_msg(1, i, d)) for i, d in enumerate(digests))
    d = hashlib.sha256(b"".join(digests)).digest()
    return el.f_bytes(1, d) + el.f_msg(el.HR_BATCH, el.f_uint(1, src) + el.f_uint(3, seq) + acks)


def test_redact_propose_step_add_results():
    # interceptor.go:219-299
    prop = el.f_msg(el.SE_PROPOSE, el.f_msg(1, request_msg(7, 9, b"secret")))
    assert el.redact_event(prop) == el.f_msg(el.SE_PROPOSE, el.f_msg(1, request_msg(7, 9, b"")))
    ack = ack_msg(3, 4, b"d" * 32)
    fwd = el.f_msg(1, ack) + el.f_bytes(2, b"payload")
    step = el.f_msg(el.SE_STEP, el.f_uint(1, 2) + el.f_msg(2, el.f_msg(14, fwd)))
    assert el.redact_event(step) == el.f_msg(el.SE_STEP, el.f_uint(1, 2) + el.f_msg(2, el.f_msg(14, el.f_msg(1, ack))))
    other_step = el.f_msg(el.SE_STEP, el.f_uint(1, 2) + el.f_msg(2, el.f_msg(15, ack)))
    assert el.redact_event(other_step) == other_step
    cp = el.f_uint(1, 20) + el.f_bytes(2, b"v")
    rr = request_result(1, 5, 6, b"abc")
    vr = verify_result(2, 5, 7, b"xyz")
    br = batch_result(0, 3, [b"a" * 32, b"b" * 32])
    ev = add_results([rr, vr, br], [cp])
    red = el.redact_event(ev)
    res = el.hash_results(red)
    assert [r.kind for r in res] == [el.HR_REQUEST, el.HR_VERIFY_REQUEST, el.HR_BATCH]
    assert [r.digest for r in res] == [r.digest for r in el.hash_results(ev)]
    assert all(r.data is None for r in res)
    assert b"abc" not in red and b"xyz" not in red and cp in red
    assert el.redact_event(red) == red  # idempotent
    assert el.redact_event(add_results([], [cp])) == add_results([], [cp])
    assert el.redact_event(TICK) == TICK


def test_recorder_redacts_unless_retained():
    ev = add_results([request_result(1, 5, 6, b"payload-bytes")])
    for retain in (False, True):
        out = io.BytesIO()
        rec = el.Recorder(3, out, time_source=lambda: 11, retain_request_data=retain)
        rec.intercept(ev)
        rec.stop()
        (got,) = list(el.Reader(io.BytesIO(out.getvalue())))
        assert got.node_id == 3 and got.time == 11
        assert (got.state_event == ev) == retain
        assert (b"payload-bytes" in got.state_event) == retain


def big_log(n_events, seed=0, level=el.DEFAULT_COMPRESSION_LEVEL):
    rng = random.Random(seed)
    out = io.BytesIO()
    t = iter(range(-5, 1 << 30))
    rec = el.Recorder(2, out, time_source=lambda: next(t), retain_request_data=True, compression_level=level)
    events = []
    for i in range(n_events):
        k = rng.randrange(4)
        if k == 0:
            ev = TICK
        elif k == 1:
            ev = add_results([request_result(i % 4, i, i * 3, rng.randbytes(rng.randrange(0, 300)))
                              for _ in range(rng.randrange(1, 6))])
        elif k == 2:
            ev = add_results([verify_result(1, i, i, rng.randbytes(40)), batch_result(1, i, [rng.randbytes(32)])])
        else:
            ev = el.f_msg(el.SE_PROPOSE, el.f_msg(1, request_msg(i, i + 1, rng.randbytes(64))))
        rec.intercept(ev)
        events.append(ev)
    rec.stop()
    return out.getvalue(), events


@pytest.mark.parametrize("level", [el.BEST_SPEED, 6, 9, -2])
def test_large_log_round_trip(level):
    data, events = big_log(3000, level=level)
    raw = gzip.decompress(data)  # independent decoder
    assert len(raw) > 4 * 65535
    got = list(el.Reader(io.BytesIO(data)))
    assert [g.state_event for g in got] == events
    assert [g.time for g in got] == list(range(-5, 3000 - 5))
    # cut mid-stream
    r = el.Reader(io.BytesIO(data[: len(data) // 2]))
    with pytest.raises(el.EventLogError):
        for _ in range(len(events) + 1):
            r.read_event()


def test_multi_member_stream():
    a, b = two_tick_log(), two_tick_log()
    assert len(list(el.Reader(io.BytesIO(a + b)))) == 4


def test_corrupt_crc_detected():
    data = bytearray(two_tick_log())
    data[-8] ^= 1
    r = el.Reader(io.BytesIO(bytes(data)))
    with pytest.raises(el.EventLogError):
        for _ in range(3):
            r.read_event()


class HashlibEngine:
    """CPU stand-in with Engine.hash_slices' signature (host logic test only)."""

    def hash_slices(self, reqs):
        return [hashlib.sha256(b"".join(r)).digest() for r in reqs]


def test_rehash_log_host_logic():
    data, events = big_log(400, seed=3)
    logged = list(el.Reader(io.BytesIO(data)))
    n, bad = el.rehash_log(logged, HashlibEngine())
    assert n > 100 and bad == []
    i = next(k for k, e in enumerate(logged) if any(r.data for r in el.hash_results(e.state_event or b"")))
    ev = logged[i].state_event
    d = el.hash_results(ev)[0].digest
    logged[i] = el.RecordedEvent(2, 0, ev.replace(d, bytes(32)))
    n2, bad2 = el.rehash_log(logged, HashlibEngine())
    assert n2 == n and bad2 == [0]


@pytest.mark.gpu
def test_rehash_log_gpu(engine):
    data, _ = big_log(2000, seed=5)
    logged = list(el.Reader(io.BytesIO(data)))
    n, bad = el.rehash_log(logged, engine)
    assert n > 1000 and bad == []
