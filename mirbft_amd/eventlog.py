"""Event-log writer/reader: the format of the reference's
``eventlog`` package, plus a re-hash of a log's recorded digests through the
engine.

Format (``eventlog/interceptor.go:301-378``): one gzip stream of records, each
``binary.PutVarint(len(msg))`` (zig-zag varint, ``:311-312``) followed by the
protobuf encoding of a ``recorderpb.RecordedEvent{node_id=1, time=2,
state_event=3}`` (``eventlog/recorderpb/recorder.proto``).  ``StateEvent`` is
kept as its encoded bytes; :func:`redact_event` and :func:`hash_results` walk
just the fields they need (``mirbftpb/mirbft.proto``: StateEvent oneof
``:394-405``, HashResult ``:408-448``, Msg ``:193-211``).

Writer compression: the reference writes through Go's ``gzip.Writer`` at
``gzip.BestSpeed`` (``interceptor.go:59,176``).  Go's BestSpeed encoder
buffers 65,535-byte windows and at ``Close`` stores a tail of <= 16 bytes, or a
tail under 128 bytes whose Huffman-only block would not save 1/16
(``compress/flate`` ``encSpeed``), as a stored block, then writes an empty
final stored block.  :class:`Recorder` does the same for any tail under 128
bytes and deflates full windows with zlib at the same level, so a log of one
small window (the reference's own 46-byte two-tick fixture,
``eventlog/interceptor_test.go:38-50``) is byte-identical to Go's, and every
log is a valid gzip stream that Go's ``gzip.Reader`` reads back (bytes differ
from Go's for larger logs; the decompressed record stream does not).
"""
from __future__ import annotations

import dataclasses
import struct
import threading
import time as _time
import zlib
from typing import BinaryIO, Callable, Iterator, List, Optional, Sequence, Tuple

from . import hashdata

BEST_SPEED = 1
DEFAULT_COMPRESSION_LEVEL = BEST_SPEED   # interceptor.go:59
DEFAULT_BUFFER_SIZE = 5000               # interceptor.go:69
_MAX_STORE_BLOCK = 65535                 # compress/flate maxStoreBlockSize
_MAX_VARINT_LEN64 = 10


class EventLogError(Exception):
    """Errors with the reference's messages (``errors.WithMessage`` chains)."""


# ---------------------------------------------------------------------------
# varints (encoding/binary) and protobuf wire format
# ---------------------------------------------------------------------------

def put_uvarint(v: int) -> bytes:
    v &= 0xFFFFFFFFFFFFFFFF
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def put_varint(v: int) -> bytes:
    """binary.PutVarint (interceptor.go:312): zig-zag, then uvarint."""
    ux = (v << 1) & 0xFFFFFFFFFFFFFFFF
    if v < 0:
        ux ^= 0xFFFFFFFFFFFFFFFF
    return put_uvarint(ux)


def read_varint(read_byte: Callable[[], Optional[int]]) -> int:
    """binary.ReadVarint (interceptor.go:359): EOFError on a clean end before the
    first byte, EventLogError('unexpected EOF') on a cut varint."""
    ux, shift = 0, 0
    for i in range(_MAX_VARINT_LEN64):
        b = read_byte()
        if b is None:
            if i == 0:
                raise EOFError
            raise EventLogError("unexpected EOF")
        if b < 0x80:
            if i == _MAX_VARINT_LEN64 - 1 and b > 1:
                raise EventLogError("binary: varint overflows a 64-bit integer")
            ux |= b << shift
            x = ux >> 1
            return ~x if ux & 1 else x
        ux |= (b & 0x7F) << shift
        shift += 7
    raise EventLogError("binary: varint overflows a 64-bit integer")


def _read_uvarint(buf: bytes, pos: int) -> Tuple[int, int]:
    v, shift = 0, 0
    while True:
        if pos >= len(buf) or shift > 63:
            raise EventLogError("could not unmarshal message: truncated varint")
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << shift
        if b < 0x80:
            return v & 0xFFFFFFFFFFFFFFFF, pos
        shift += 7


def parse_fields(buf: bytes) -> List[Tuple[int, int, object]]:
    """Protobuf wire fields in order: (number, wire type, int | bytes)."""
    out, pos = [], 0
    while pos < len(buf):
        key, pos = _read_uvarint(buf, pos)
        num, wt = key >> 3, key & 7
        if num == 0:
            raise EventLogError("could not unmarshal message: invalid field number")
        if wt == 0:
            v, pos = _read_uvarint(buf, pos)
        elif wt == 1:
            v, pos = bytes(buf[pos:pos + 8]), pos + 8
        elif wt == 2:
            n, pos = _read_uvarint(buf, pos)
            v, pos = bytes(buf[pos:pos + n]), pos + n
        elif wt == 5:
            v, pos = bytes(buf[pos:pos + 4]), pos + 4
        else:
            raise EventLogError("could not unmarshal message: unsupported wire type %d" % wt)
        if pos > len(buf):
            raise EventLogError("could not unmarshal message: unexpected EOF")
        out.append((num, wt, v))
    return out


def _key(num: int, wt: int) -> bytes:
    return put_uvarint((num << 3) | wt)


def f_uint(num: int, v: int) -> bytes:
    """A proto3 scalar varint field (omitted when zero)."""
    return _key(num, 0) + put_uvarint(v) if v else b""


def f_bytes(num: int, v: bytes) -> bytes:
    """A proto3 bytes field (omitted when empty)."""
    return _key(num, 2) + put_uvarint(len(v)) + v if v else b""


def f_msg(num: int, v: Optional[bytes]) -> bytes:
    """A message field: present (even when empty) unless None."""
    return b"" if v is None else _key(num, 2) + put_uvarint(len(v)) + v


def _get(fields, num: int, default=None):
    """Last value of field `num` (proto3 last-one-wins), or default."""
    v = default
    for n, _, x in fields:
        if n == num:
            v = x
    return v


def _oneof(fields, nums) -> Tuple[Optional[int], object]:
    which, val = None, None
    for n, _, x in fields:
        if n in nums:
            which, val = n, x
    return which, val


# ---------------------------------------------------------------------------
# messages
# ---------------------------------------------------------------------------

# StateEvent oneof numbers (mirbft.proto:394-405)
SE_INITIALIZE, SE_LOAD_ENTRY, SE_LOAD_REQUEST, SE_COMPLETE_INIT, SE_ADD_RESULTS = 1, 2, 3, 4, 5
SE_TRANSFER, SE_PROPOSE, SE_STEP, SE_TICK, SE_ACTIONS_RECEIVED = 6, 7, 8, 9, 10
_SE_TYPES = frozenset(range(1, 11))
# HashResult oneof numbers (mirbft.proto:441-447)
HR_REQUEST, HR_BATCH, HR_EPOCH_CHANGE, HR_VERIFY_BATCH, HR_VERIFY_REQUEST = 2, 3, 4, 5, 6
_HR_TYPES = frozenset(range(2, 7))
_MSG_FORWARD_REQUEST = 14   # Msg oneof (mirbft.proto:208)


def tick_event() -> bytes:
    """StateEvent{Tick: &TickElapsed{}} (interceptor_test.go:23-27)."""
    return f_msg(SE_TICK, b"")


@dataclasses.dataclass(frozen=True)
class RecordedEvent:
    """recorderpb.RecordedEvent; ``state_event`` is the encoded StateEvent (None: unset)."""
    node_id: int = 0
    time: int = 0
    state_event: Optional[bytes] = None

    def marshal(self) -> bytes:
        return f_uint(1, self.node_id) + f_uint(2, self.time & 0xFFFFFFFFFFFFFFFF) + f_msg(3, self.state_event)

    @classmethod
    def unmarshal(cls, buf: bytes) -> "RecordedEvent":
        fields = parse_fields(buf)
        t = _get(fields, 2, 0)
        if t >= 1 << 63:
            t -= 1 << 64
        return cls(node_id=_get(fields, 1, 0), time=t, state_event=_get(fields, 3))


def _redact_request(req: bytes) -> bytes:
    f = parse_fields(req)
    return f_uint(1, _get(f, 1, 0)) + f_uint(2, _get(f, 2, 0))


def redact_event(event: bytes) -> bytes:
    """interceptor.go:219-299: drop request payloads from Propose, Step/ForwardRequest
    and the Request / VerifyRequest hash results of AddResults; everything else
    is returned as is."""
    fields = parse_fields(event)
    which, val = _oneof(fields, _SE_TYPES)
    if which == SE_PROPOSE:                                   # :221-231
        req = _get(parse_fields(val), 1, b"")
        return f_msg(SE_PROPOSE, f_msg(1, _redact_request(req)))
    if which == SE_STEP:                                      # :232-250
        step = parse_fields(val)
        msg = _get(step, 2, b"")
        mw, mv = _oneof(parse_fields(msg), range(1, 16))
        if mw == _MSG_FORWARD_REQUEST:
            ack = _get(parse_fields(mv), 1)
            fwd = f_msg(1, ack)
            return f_msg(SE_STEP, f_uint(1, _get(step, 1, 0)) + f_msg(2, f_msg(_MSG_FORWARD_REQUEST, fwd)))
        return event
    if which == SE_ADD_RESULTS:                               # :251-295
        res = parse_fields(val)
        digests = [v for n, _, v in res if n == 1]
        if not digests:
            return event
        out = bytearray()
        for hr in digests:
            hf = parse_fields(hr)
            digest = _get(hf, 1, b"")
            hw, hv = _oneof(hf, _HR_TYPES)
            if hw == HR_REQUEST:
                rf = parse_fields(hv)
                body = f_uint(1, _get(rf, 1, 0)) + f_msg(2, _redact_request(_get(rf, 2, b"")))
                hr = f_bytes(1, digest) + f_msg(HR_REQUEST, body)
            elif hw == HR_VERIFY_REQUEST:
                vf = parse_fields(hv)
                body = f_uint(1, _get(vf, 1, 0)) + f_msg(2, _get(vf, 2))
                hr = f_bytes(1, digest) + f_msg(HR_VERIFY_REQUEST, body)
            out += f_msg(1, hr)
        for n, _, v in res:
            if n == 2:
                out += f_msg(2, v)
        return f_msg(SE_ADD_RESULTS, bytes(out))
    return event


@dataclasses.dataclass(frozen=True)
class LoggedHashResult:
    """One HashResult of an AddResults event: its oneof kind, the digest the
    processor produced and, for Request / VerifyRequest results whose log kept
    the payload (RetainRequestDataOpt), the ``[][]byte`` it hashed."""
    kind: int
    digest: bytes
    data: Optional[List[bytes]] = None


def hash_results(event: bytes) -> List[LoggedHashResult]:
    """The digests of an AddResults StateEvent (empty for other events).  Data
    layouts: request state_machine.go:313-317, VerifyRequest
    client_tracker.go:618-622 (hashdata.request_hash_data)."""
    which, val = _oneof(parse_fields(event), _SE_TYPES)
    if which != SE_ADD_RESULTS:
        return []
    out = []
    for n, _, hr in parse_fields(val):
        if n != 1:
            continue
        hf = parse_fields(hr)
        hw, hv = _oneof(hf, _HR_TYPES)
        data = None
        if hw == HR_REQUEST:
            req = parse_fields(_get(parse_fields(hv), 2, b""))
            payload = _get(req, 3, b"")
            if payload:
                data = hashdata.request_hash_data(_get(req, 1, 0), _get(req, 2, 0), payload)
        elif hw == HR_VERIFY_REQUEST:
            vf = parse_fields(hv)
            payload = _get(vf, 3, b"")
            if payload:
                ack = parse_fields(_get(vf, 2, b""))
                data = hashdata.request_hash_data(_get(ack, 1, 0), _get(ack, 2, 0), payload)
        out.append(LoggedHashResult(kind=hw or 0, digest=_get(hf, 1, b""), data=data))
    return out


def rehash_log(events: Sequence[RecordedEvent], engine) -> Tuple[int, List[int]]:
    """Re-hash every payload-carrying Request / VerifyRequest result of a log in
    ONE engine call (``Engine.hash_slices``) and compare with the recorded
    digests.  Returns (results checked, indices of mismatches)."""
    todo = [r for ev in events if ev.state_event for r in hash_results(ev.state_event) if r.data is not None]
    if not todo:
        return 0, []
    got = engine.hash_slices([r.data for r in todo])
    bad = [i for i, r in enumerate(todo) if bytes(got[i]) != r.digest]
    return len(todo), bad


# ---------------------------------------------------------------------------
# writer
# ---------------------------------------------------------------------------

def _stored_block(data: bytes, final: bool) -> bytes:
    n = len(data)
    return bytes([1 if final else 0]) + struct.pack("<HH", n, n ^ 0xFFFF) + data


class _GzipWriter:
    """gzip member in Go's layout: header 1f8b 08 00 mtime=0 xfl os=255."""

    def __init__(self, dest: BinaryIO, level: int):
        if not (-2 <= level <= 9):
            raise EventLogError("gzip: invalid compression level: %d" % level)
        self.dest, self.level = dest, level
        xfl = 4 if level == BEST_SPEED else (2 if level == 9 else 0)
        dest.write(b"\x1f\x8b\x08\x00\x00\x00\x00\x00" + bytes([xfl, 255]))
        strategy = zlib.Z_HUFFMAN_ONLY if level == -2 else zlib.Z_DEFAULT_STRATEGY
        self._z = zlib.compressobj(max(level, -1) if level != -2 else 1, zlib.DEFLATED, -15, 8, strategy)
        self._win = bytearray()
        self._crc, self._size = 0, 0

    def write(self, b: bytes) -> None:
        self._crc = zlib.crc32(b, self._crc)
        self._size += len(b)
        self._win += b
        while len(self._win) >= _MAX_STORE_BLOCK:
            chunk = bytes(self._win[:_MAX_STORE_BLOCK])
            del self._win[:_MAX_STORE_BLOCK]
            self.dest.write(self._z.compress(chunk) + self._z.flush(zlib.Z_SYNC_FLUSH))

    def close(self) -> None:
        tail = bytes(self._win)
        self._win.clear()
        if tail and len(tail) < 128 and self.level == BEST_SPEED:
            self.dest.write(_stored_block(tail, False))
        elif tail:
            self.dest.write(self._z.compress(tail) + self._z.flush(zlib.Z_SYNC_FLUSH))
        self.dest.write(_stored_block(b"", True))
        self.dest.write(struct.pack("<II", self._crc & 0xFFFFFFFF, self._size & 0xFFFFFFFF))


def write_recorded_event(writer, event: RecordedEvent) -> None:
    """WriteRecordedEvent / writeSizePrefixedProto (interceptor.go:301-322)."""
    msg = event.marshal()
    writer.write(put_varint(len(msg)))
    writer.write(msg)


class Recorder:
    """eventlog.Recorder (interceptor.go:84-217), an EventInterceptor:
    ``intercept(state_event)`` stamps the event with ``time_source()``, redacts it
    unless ``retain_request_data`` and appends it to the gzip stream on ``dest``;
    ``stop()`` finishes the stream.  Writes happen on the caller's thread (the
    reference's goroutine + ``buffer_size`` channel only decouple the state
    machine from the writer), under a lock."""

    def __init__(self, node_id: int, dest: BinaryIO, time_source: Optional[Callable[[], int]] = None,
                 retain_request_data: bool = False, compression_level: int = DEFAULT_COMPRESSION_LEVEL,
                 buffer_size: int = DEFAULT_BUFFER_SIZE):
        start = _time.monotonic()
        self.node_id = node_id
        self.time_source = time_source or (lambda: int((_time.monotonic() - start) * 1000))
        self.retain_request_data = retain_request_data
        self.buffer_size = buffer_size
        self._gz = _GzipWriter(dest, compression_level)
        self._lock = threading.Lock()
        self._stopped = False

    def intercept(self, state_event: bytes) -> None:
        t = self.time_source()
        with self._lock:
            if self._stopped:
                raise EventLogError("interceptor stopped at caller request")
            ev = state_event if self.retain_request_data else redact_event(state_event)
            write_recorded_event(self._gz, RecordedEvent(self.node_id, t, ev))

    def stop(self) -> None:
        with self._lock:
            if not self._stopped:
                self._stopped = True
                self._gz.close()


# ---------------------------------------------------------------------------
# reader
# ---------------------------------------------------------------------------

class _GzipStream:
    """Incremental gzip decode of a byte source (multi-member, CRC checked)."""

    def __init__(self, source: BinaryIO):
        self.src = source
        self.buf = bytearray()
        self.pos = 0
        self._z = None
        self._raw = b""
        self._eof = False
        head = self._src_read_exact(10)
        if len(head) < 10:   # Go: io.EOF on an empty source, io.ErrUnexpectedEOF on a cut header
            raise EventLogError("could not read source as a gzip stream: %s" % ("unexpected EOF" if head else "EOF"))
        if head[:2] != b"\x1f\x8b" or head[2] != 8:
            raise EventLogError("could not read source as a gzip stream: gzip: invalid header")
        self._start_member(head)

    def _src_read_exact(self, n: int) -> bytes:
        out = bytearray(self._raw[:n])
        self._raw = self._raw[n:]
        while len(out) < n:
            b = self.src.read(n - len(out))
            if not b:
                break
            out += b
        return bytes(out)

    def _start_member(self, head: bytes) -> None:
        flg = head[3]
        hdr = bytearray(head)
        if flg & 4:   # FEXTRA
            xl = self._src_read_exact(2)
            hdr += xl + self._src_read_exact(struct.unpack("<H", xl)[0] if len(xl) == 2 else 0)
        for bit in (8, 16):   # FNAME, FCOMMENT: zero-terminated
            if flg & bit:
                while True:
                    c = self._src_read_exact(1)
                    hdr += c
                    if not c or c == b"\x00":
                        break
        if flg & 2:
            hdr += self._src_read_exact(2)
        # Feed the whole header back to a gzip-mode decompressor (checks CRC/size).
        self._z = zlib.decompressobj(31)
        self._pending_head = bytes(hdr)

    def _fill(self) -> bool:
        """Decode more bytes into buf; False at the end of the last member."""
        while True:
            if self._eof:
                return False
            if self._pending_head is not None:
                data, self._pending_head = self._pending_head, None
            else:
                data = self._raw or self.src.read(1 << 16)
                self._raw = b""
            if not data:
                if not self._z.eof:
                    raise EventLogError("unexpected EOF")
                self._eof = True
                return False
            try:
                out = self._z.decompress(data)
            except zlib.error as e:
                raise EventLogError("gzip: %s" % e) from None
            if self._z.eof:
                rest = self._z.unused_data
                # next member, if any
                nxt = rest + (self.src.read(10 - len(rest)) if len(rest) < 10 else b"")
                if nxt:
                    if len(nxt) < 10 or nxt[:2] != b"\x1f\x8b":
                        raise EventLogError("gzip: invalid header")
                    self._raw = nxt[10:]
                    self._start_member(nxt[:10])
                else:
                    self._eof = True
            if out:
                if self.pos:
                    del self.buf[:self.pos]
                    self.pos = 0
                self.buf += out
                return True

    def read_byte(self) -> Optional[int]:
        if self.pos >= len(self.buf) and not self._fill():
            return None
        b = self.buf[self.pos]
        self.pos += 1
        return b

    def read(self, n: int) -> bytes:
        while len(self.buf) - self.pos < n and self._fill():
            pass
        out = bytes(self.buf[self.pos:self.pos + n])
        self.pos += len(out)
        return out


class Reader:
    """eventlog.Reader (interceptor.go:324-378).  ``read_event()`` returns the
    next RecordedEvent and raises EOFError after the last one (Go: io.EOF);
    other failures raise EventLogError with the reference's messages."""

    def __init__(self, source: BinaryIO):
        self._s = _GzipStream(source)

    def read_event(self) -> RecordedEvent:
        try:
            n = read_varint(self._s.read_byte)
        except EOFError:
            raise
        except EventLogError as e:
            raise EventLogError("error reading event: could not read size prefix: %s" % e) from None
        if n < 0:
            raise EventLogError("error reading event: could not read size prefix: negative length %d" % n)
        try:
            msg = self._s.read(n)
        except EventLogError as e:
            raise EventLogError("error reading event: could not read message: %s" % e) from None
        if len(msg) < n:
            raise EventLogError("error reading event: could not read message: EOF")
        try:
            return RecordedEvent.unmarshal(msg)
        except EventLogError as e:
            raise EventLogError("error reading event: %s" % e) from None

    def __iter__(self) -> Iterator[RecordedEvent]:
        while True:
            try:
                yield self.read_event()
            except EOFError:
                return
