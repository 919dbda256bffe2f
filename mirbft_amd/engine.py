"""Engine: one gfx950 device context behind the C-ABI (include/mirsha.h).

Host-memory entry points take numpy arrays / bytes and return numpy digests
``(n, 32) uint8`` in ORIGIN order.  Device-pointer entry points take raw device
addresses (ints, e.g. ``torch.Tensor.data_ptr()``) and are asynchronous on the
engine's stream.  Every call runs the HIP kernels; there is no CPU path here.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Sequence

import numpy as np

from . import _lib
from ._lib import MIRSHA_NULL_INDEX, MirshaError, check

KERNEL_MSGS = 0
KERNEL_LISTS = 1
KERNEL_GEN = 2
KERNEL_CHAIN = 3
KERNEL_FUSED = 4
KERNEL_OVERLAP = 5
ASYNC_SLOTS = 4  # submissions in flight per context (mirsha_submit_slices)

# mirsha_pipeline modes (include/mirsha.h)
PIPELINE_SEQUENTIAL = 0
PIPELINE_FUSED = 1
PIPELINE_AUTO = 3
PIPELINE_MODES = {"sequential": PIPELINE_SEQUENTIAL, "fused": PIPELINE_FUSED, "auto": PIPELINE_AUTO}
VARIANT_LDS = 0
VARIANT_DIRECT = 1
VARIANT_LOWOCC = 4
VARIANT_LDS_ONLY = 5
VARIANT_PAIR = 6
VARIANT_CU = 10
VARIANTS = (VARIANT_LDS, VARIANT_DIRECT, VARIANT_LOWOCC, VARIANT_LDS_ONLY, VARIANT_PAIR, VARIANT_CU)


def _ptr(a: np.ndarray | None) -> int | None:
    if a is None:
        return None
    return a.ctypes.data if a.size else None


def _as_u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf.reshape(-1).view(np.uint8))
    return np.frombuffer(memoryview(buf), dtype=np.uint8)


class SliceArrays:
    """HashRequest.Data of n requests as the C-ABI's slice arrays: slice s is
    ``len[s]`` bytes at address ``ptr[s]``; request i = slices [first[i], first[i+1]).
    Holds references to the Python buffers the pointers come from."""

    def __init__(self, ptr: np.ndarray, length: np.ndarray, first: np.ndarray, keep=()):
        self.ptr = np.ascontiguousarray(ptr, dtype=np.uint64)
        self.len = np.ascontiguousarray(length, dtype=np.uint64)
        self.first = np.ascontiguousarray(first, dtype=np.uint32)
        if self.ptr.shape != self.len.shape or self.first.size < 1 or int(self.first[-1]) != self.ptr.size:
            raise ValueError("inconsistent slice arrays")
        self.keep = keep
        self.n = int(self.first.size) - 1
        self.ptr_p = _ptr(self.ptr)
        self.len_p = _ptr(self.len)
        self.first_p = _ptr(self.first)

    @classmethod
    def from_requests(cls, requests: Sequence[Sequence[bytes]]) -> "SliceArrays":
        keep, lens, first = [], [], [0]
        for req in requests:
            for s in req:
                b = bytes(s)
                keep.append(b)
                lens.append(len(b))
            first.append(len(keep))
        ptr = np.zeros(len(keep), dtype=np.uint64)
        for i, b in enumerate(keep):
            if len(b):
                ptr[i] = ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value
        return cls(ptr, np.asarray(lens, dtype=np.uint64), np.asarray(first, dtype=np.uint32), keep)

    @classmethod
    def from_buffer(cls, buf: np.ndarray, slice_off: np.ndarray, slice_len: np.ndarray, first: np.ndarray):
        """Slices that are byte ranges of one numpy buffer (vectorised; for large streams)."""
        b = np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
        base = b.ctypes.data
        off = np.ascontiguousarray(slice_off, dtype=np.uint64)
        return cls(np.uint64(base) + off, slice_len, first, (b,))


class Ticket:
    """A submission of Engine.submit_slices; ``out`` receives the digests."""

    def __init__(self, value: int, out: np.ndarray):
        self.value = value
        self.out = out


def _out_rows(out, n: int) -> np.ndarray:
    """A caller-supplied (n, 32) uint8 result array (checked), or a new one."""
    if out is None:
        return np.empty((n, 32), dtype=np.uint8)
    if not isinstance(out, np.ndarray) or out.dtype != np.uint8 or out.shape != (n, 32) or not out.flags.c_contiguous \
            or not out.flags.writeable:
        raise ValueError(f"out must be a writeable C-contiguous uint8 array of shape ({n}, 32)")
    return out


def dedup_plan(requests) -> tuple[np.ndarray, int]:
    """Host-only dedup plan (mirsha_dedup_plan): rep[i] = smallest j <= i with
    identical request bytes; returns (rep, number of distinct requests)."""
    sl = requests if isinstance(requests, SliceArrays) else SliceArrays.from_requests(requests)
    rep = np.empty(sl.n, dtype=np.uint32)
    u = ctypes.c_uint32(0)
    rc = _lib.load().mirsha_dedup_plan(sl.ptr_p, sl.len_p, sl.first_p, sl.n, _ptr(rep), ctypes.byref(u))
    check(rc)
    return rep, u.value


def device_count() -> int:
    n = ctypes.c_int(0)
    check(_lib.load().mirsha_device_count(ctypes.byref(n)))
    return n.value


class Engine:
    """Batched SHA-256 engine on one MI355X.  Replaces `Hasher` (processor.go:21)."""

    def __init__(self, device: int = 0):
        self._lib = _lib.load()
        ctx = ctypes.c_void_p()
        rc = self._lib.mirsha_ctx_create(int(device), ctypes.byref(ctx))
        if rc != 0:
            raise MirshaError(rc, f"cannot create a gfx950 context on device {device}")
        self.ctx = ctx
        self.device = device
        self.last_unique = 0
        # Output arrays of submissions the library has not retired yet: it
        # writes the digests there inside mirsha_wait / mirsha_poll, or when a
        # later submit retires the oldest of its ASYNC_SLOTS ring slots, so
        # they must outlive a dropped Ticket.
        self._outstanding: dict[int, np.ndarray] = {}

    # ------------------------------------------------------------ lifecycle
    def close(self) -> None:
        if getattr(self, "ctx", None):
            self._lib.mirsha_ctx_destroy(self.ctx)  # no digest is written after this
            self.ctx = None
            self._outstanding = {}

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int) -> None:
        check(rc, self.ctx)

    # --------------------------------------------------------------- knobs
    def set_stream(self, stream_ptr: int | None) -> None:
        self._check(self._lib.mirsha_ctx_set_stream(self.ctx, stream_ptr))

    @property
    def stream(self) -> int:
        return self._lib.mirsha_ctx_stream(self.ctx) or 0

    def set_variant(self, variant: int) -> None:
        self._check(self._lib.mirsha_ctx_set_variant(self.ctx, int(variant)))

    def set_timing(self, enable: bool) -> None:
        self._check(self._lib.mirsha_ctx_set_timing(self.ctx, 1 if enable else 0))

    def kernel_time(self, kernel: int) -> tuple[int, float]:
        n = ctypes.c_uint64(0)
        ms = ctypes.c_double(0.0)
        self._check(self._lib.mirsha_ctx_kernel_time(self.ctx, int(kernel), ctypes.byref(n), ctypes.byref(ms)))
        return n.value, ms.value

    def set_timing_mask(self, kernels) -> None:
        """Time only these kernel ids (KERNEL_*) while timing is enabled."""
        m = 0
        for k in kernels:
            m |= 1 << int(k)
        self._check(self._lib.mirsha_ctx_set_timing_mask(self.ctx, m))

    def reset_timing(self) -> None:
        self._check(self._lib.mirsha_ctx_reset_timing(self.ctx))

    def sync(self) -> None:
        self._check(self._lib.mirsha_sync(self.ctx))

    # ------------------------------------------------------------ host API
    def hash_batch(self, arena, off: Sequence[int], length: Sequence[int], out=None) -> np.ndarray:
        """Digest of arena[off[i]:off[i]+len[i]] for every i (processor.go:133-143).
        out: optional reusable uint8 (n, 32) result array."""
        a = _as_u8(arena)
        o = np.ascontiguousarray(off, dtype=np.uint64)
        ln = np.ascontiguousarray(length, dtype=np.uint32)
        if o.shape != ln.shape:
            raise ValueError("off and len differ in length")
        n = int(o.size)
        out = _out_rows(out, n)
        if n:
            self._check(self._lib.mirsha_hash_batch(self.ctx, _ptr(a), a.size, _ptr(o), _ptr(ln), n, _ptr(out)))
        return out

    def hash_messages(self, messages: Sequence[bytes]) -> np.ndarray:
        """One digest per message (each a single byte string)."""
        lens = np.fromiter((len(m) for m in messages), dtype=np.uint32, count=len(messages))
        off = np.zeros(len(messages), dtype=np.uint64)
        if len(messages) > 1:
            np.cumsum(lens[:-1], out=off[1:])
        arena = b"".join(messages)
        return self.hash_batch(arena, off, lens)

    def hash_slices(self, requests: Sequence[Sequence[bytes]], dedup: bool = False) -> np.ndarray:
        """Digest of concat(req) for each req = HashRequest.Data (actions.go:157-164).
        dedup=True hashes each distinct content once (mirsha_hash_slices_dedup);
        ``self.last_unique`` then holds the number of distinct requests."""
        sl = SliceArrays.from_requests(requests)
        return self.hash_slice_arrays(sl, dedup)

    def hash_slice_arrays(self, sl: "SliceArrays", dedup: bool = False) -> np.ndarray:
        """hash_slices over prepared slice arrays (pointer / length / first)."""
        n = sl.n
        out = np.empty((n, 32), dtype=np.uint8)
        if n == 0:
            self.last_unique = 0
            return out
        if dedup:
            u = ctypes.c_uint32(0)
            self._check(self._lib.mirsha_hash_slices_dedup(self.ctx, sl.ptr_p, sl.len_p, sl.first_p, n, _ptr(out),
                                                           ctypes.byref(u)))
            self.last_unique = u.value
        else:
            self._check(self._lib.mirsha_hash_slices(self.ctx, sl.ptr_p, sl.len_p, sl.first_p, n, _ptr(out)))
            self.last_unique = n
        return out

    def host_empty(self, nbytes: int) -> np.ndarray:
        """A uint8 array in page-locked host memory (mirsha_host_alloc), freed
        with the array: the caller's arena at PCIe rate."""
        p = ctypes.c_void_p()
        self._check(self._lib.mirsha_host_alloc(self.ctx, int(nbytes), ctypes.byref(p)))
        buf = (ctypes.c_uint8 * max(int(nbytes), 1)).from_address(p.value)
        arr = np.frombuffer(buf, dtype=np.uint8, count=int(nbytes))
        import weakref

        weakref.finalize(buf, self._lib.mirsha_host_free, p.value)
        return arr

    def submit_slices(self, requests, dedup: bool = False) -> "Ticket":
        """Asynchronous, order-preserving submission (mirsha_submit_slices): the
        requests are packed before this returns; ``wait(ticket)`` yields the
        digests in origin order.  ``requests`` may be a list of slice lists or
        a SliceArrays."""
        sl = requests if isinstance(requests, SliceArrays) else SliceArrays.from_requests(requests)
        out = np.empty((sl.n, 32), dtype=np.uint8)
        t = ctypes.c_uint64(0)
        self._check(self._lib.mirsha_submit_slices(self.ctx, sl.ptr_p, sl.len_p, sl.first_p, sl.n, _ptr(out),
                                                   _lib.MIRSHA_SUBMIT_DEDUP if dedup else 0, ctypes.byref(t)))
        self._outstanding[t.value] = out
        # Submission t took the ring slot of t - ASYNC_SLOTS, which the library
        # completed (in order) before reusing it.
        self._retire(t.value - ASYNC_SLOTS)
        return Ticket(t.value, out)

    def submit_batch(self, arena, off, length, out=None) -> "Ticket":
        """Asynchronous arena submission (mirsha_submit_batch, the Go binding's
        chunked HashBatch): request i = arena[off[i]:off[i]+len[i]].  A
        page-locked arena (host_empty) is DMA'd from in place and must not
        change until the ticket is waited for; a page-locked ``out`` receives
        the digests by DMA."""
        a = _as_u8(arena)
        o = np.ascontiguousarray(off, dtype=np.uint64)
        ln = np.ascontiguousarray(length, dtype=np.uint32)
        if o.shape != ln.shape:
            raise ValueError("off and len differ in length")
        n = int(o.size)
        out = _out_rows(out, n)
        t = ctypes.c_uint64(0)
        self._check(self._lib.mirsha_submit_batch(self.ctx, _ptr(a), a.size, _ptr(o), _ptr(ln), n, _ptr(out),
                                                  ctypes.byref(t)))
        self._outstanding[t.value] = (out, a)  # the arena too: it may be read until the ticket retires
        self._retire(t.value - ASYNC_SLOTS)
        return Ticket(t.value, out)

    def _retire(self, upto: int) -> None:
        for k in [k for k in self._outstanding if k <= upto]:
            del self._outstanding[k]

    def wait(self, ticket: "Ticket") -> np.ndarray:
        self._check(self._lib.mirsha_wait(self.ctx, ticket.value))
        self._retire(ticket.value)
        return ticket.out

    def poll(self, ticket: "Ticket") -> bool:
        done = ctypes.c_int(0)
        self._check(self._lib.mirsha_poll(self.ctx, ticket.value, ctypes.byref(done)))
        if done.value:
            self._retire(ticket.value)
        return bool(done.value)

    def hash_requests_then_batches(self, arena, off, length, idx, batch_first, out=None, batch_out=None):
        """Request digests, then batch digests over them on device (sequence.go:154-157).

        out / batch_out: optional C-contiguous uint8 (n, 32) / (n_batches, 32)
        arrays reused across calls.  A fresh 32 MiB result array costs ~30 ms
        of first-touch page faults per call (glibc hands large allocations
        out as new mmaps), which is more than the GPU work at 1M requests."""
        a = _as_u8(arena)
        o = np.ascontiguousarray(off, dtype=np.uint64)
        ln = np.ascontiguousarray(length, dtype=np.uint32)
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        fs = np.ascontiguousarray(batch_first, dtype=np.uint32)
        n, nb = int(o.size), int(fs.size) - 1
        if nb < 0:
            raise ValueError("batch_first needs n_batches + 1 entries")
        req = _out_rows(out, n)
        bat = _out_rows(batch_out, nb)
        self._check(
            self._lib.mirsha_hash_requests_then_batches(
                self.ctx, _ptr(a), a.size, _ptr(o), _ptr(ln), n, _ptr(ix), _ptr(fs), nb, _ptr(req), _ptr(bat)
            )
        )
        return req, bat

    def digest_lists(self, digests, idx, list_first) -> np.ndarray:
        """SHA-256 over ordered lists of 32-byte digests (batch / VerifyBatch / checkpoint chain)."""
        d = np.ascontiguousarray(digests, dtype=np.uint8).reshape(-1, 32)
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        fs = np.ascontiguousarray(list_first, dtype=np.uint32)
        nl = int(fs.size) - 1
        out = np.empty((max(nl, 0), 32), dtype=np.uint8)
        if nl > 0:
            self._check(
                self._lib.mirsha_digest_lists(self.ctx, _ptr(d), d.shape[0], _ptr(ix), _ptr(fs), nl, _ptr(out))
            )
        return out

    # ---------------------------------------------------------- device API
    def hash_batch_device(self, d_arena: int, arena_len: int, d_off: int, d_len: int, d_order: int | None,
                          n: int, d_out: int) -> None:
        self._check(self._lib.mirsha_hash_batch_device(self.ctx, d_arena, arena_len, d_off, d_len, d_order, n, d_out))

    def digest_lists_device(self, d_digests: int, n_digests: int, d_idx: int, d_first: int, n_lists: int,
                            n_entries: int, d_out: int) -> None:
        self._check(self._lib.mirsha_digest_lists_device(self.ctx, d_digests, n_digests, d_idx, d_first, n_lists,
                                                         n_entries, d_out))

    def pipeline(self, n_req: int, idx, list_first, length=None, mode: int | str | None = None) -> "Pipeline":
        """Plan for request -> batch-digest runs with this list shape (host index lists).
        mode: PIPELINE_AUTO (default) / _FUSED / _SEQUENTIAL or its name."""
        return Pipeline(self, n_req, idx, list_first, length, mode)

    def hash_requests_then_batches_device(self, plan: "Pipeline", d_arena: int, arena_len: int, d_off: int,
                                          d_len: int, d_req_out: int, d_batch_out: int) -> None:
        self._check(self._lib.mirsha_hash_requests_then_batches_device(
            self.ctx, plan.handle, d_arena, arena_len, d_off, d_len, d_req_out, d_batch_out))

    def pipeline_overlap_device(self, plan: "Pipeline", d_arena: int, arena_len: int, d_off: int, d_len: int,
                                d_req_out: int, d_prev_req: int, d_prev_batch_out: int) -> None:
        """One launch: this cycle's requests -> d_req_out and the previous cycle's
        batch digests from d_prev_req -> d_prev_batch_out (0 = none; see mirsha.h)."""
        self._check(self._lib.mirsha_pipeline_overlap_device(
            self.ctx, plan.handle, d_arena or None, arena_len, d_off or None, d_len or None, d_req_out or None,
            d_prev_req or None, d_prev_batch_out or None))

    def synth_requests_device(self, seed: int, first: int, count: int, data_len: int, d_arena: int) -> None:
        self._check(self._lib.mirsha_synth_requests_device(self.ctx, seed, first, count, data_len, d_arena))

    def synth_mixed_lengths_device(self, seed: int, first: int, count: int, d_len: int) -> None:
        """Config-5 message lengths (u32) of requests [first, first + count) into d_len."""
        self._check(self._lib.mirsha_synth_mixed_lengths_device(self.ctx, seed, first, count, d_len))

    def synth_mixed_device(self, seed: int, first: int, count: int, d_off: int, d_arena: int) -> None:
        """Config-5 message bytes of requests [first, first + count) at d_arena + d_off[r]."""
        self._check(self._lib.mirsha_synth_mixed_device(self.ctx, seed, first, count, d_off, d_arena))

    HOST_PHASES = ("validate", "plan", "pack", "device", "scatter", "total", "chunks")

    def host_profile(self) -> dict:
        """Host-side phases (ms) of the last slice submission (mirsha_ctx_host_profile)."""
        buf = (ctypes.c_double * len(self.HOST_PHASES))()
        n = self._lib.mirsha_ctx_host_profile(self.ctx, buf, len(self.HOST_PHASES))
        if n < 0:
            self._check(n)
        return {k: buf[i] for i, k in enumerate(self.HOST_PHASES)}

    def clock_probe(self, iters: int = 128) -> tuple[float, float]:
        """(clock GHz held under the compression load, SIMD cycles per 64-lane
        compression with no memory traffic): mirsha_clock_probe."""
        ghz, cyc = ctypes.c_double(0.0), ctypes.c_double(0.0)
        self._check(self._lib.mirsha_clock_probe(self.ctx, int(iters), ctypes.byref(ghz), ctypes.byref(cyc)))
        return ghz.value, cyc.value


class Pipeline:
    """mirsha_pipeline: a request -> batch-digest plan reused across runs of one
    shape (see include/mirsha.h for the modes)."""

    def __init__(self, engine: Engine, n_req: int, idx, list_first, length=None, mode=None):
        self._lib = engine._lib
        self._engine = engine
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        fs = np.ascontiguousarray(list_first, dtype=np.uint32)
        ln = None if length is None else np.ascontiguousarray(length, dtype=np.uint32)
        h = ctypes.c_void_p()
        if mode is None:
            engine._check(self._lib.mirsha_pipeline_create(engine.ctx, int(n_req), _ptr(ln), _ptr(ix), _ptr(fs),
                                                           int(fs.size) - 1, ctypes.byref(h)))
        else:
            m = PIPELINE_MODES[mode] if isinstance(mode, str) else int(mode)
            engine._check(self._lib.mirsha_pipeline_create_mode(engine.ctx, int(n_req), _ptr(ln), _ptr(ix),
                                                                _ptr(fs), int(fs.size) - 1, m, ctypes.byref(h)))
        self.handle = h
        self.mode = int(self._lib.mirsha_pipeline_mode(h))
        # 1: a fused plan built sequential after its placement probe (mirsha_pipeline_fallback)
        self.fallback = int(self._lib.mirsha_pipeline_fallback(h)) if hasattr(self._lib, "mirsha_pipeline_fallback") \
            else 0
        self.n_req = int(n_req)
        self.n_lists = int(fs.size) - 1

    @property
    def mode_name(self) -> str:
        return {v: k for k, v in PIPELINE_MODES.items()}[self.mode]

    def status(self) -> None:
        """Synchronise and raise if a fused run's readiness watchdog expired."""
        self._engine._check(self._lib.mirsha_pipeline_status(self._engine.ctx, self.handle))

    def shape(self) -> tuple[int, int, int]:
        """(n_tiles, n_counters, n_groups) of a fused plan."""
        t, c, g = ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_uint32(0)
        check(self._lib.mirsha_pipeline_shape(self.handle, ctypes.byref(t), ctypes.byref(c), ctypes.byref(g)))
        return t.value, c.value, g.value

    def split_tiles(self) -> tuple[int, int]:
        """(split tiles, segments per tile) of a fused plan (mirsha_pipeline_split_tiles)."""
        n, k = ctypes.c_uint32(0), ctypes.c_uint32(0)
        check(self._lib.mirsha_pipeline_split_tiles(self.handle, ctypes.byref(n), ctypes.byref(k)))
        return n.value, k.value

    def trace(self) -> np.ndarray | None:
        """Last run's fused timeline (MIRSHA_FUSED_TRACE=1 at plan creation), see include/mirsha.h."""
        n = ctypes.c_uint64(0)
        self._engine._check(self._lib.mirsha_pipeline_trace(self._engine.ctx, self.handle, None, 0, ctypes.byref(n)))
        if n.value == 0:
            return None
        out = np.zeros(n.value, dtype=np.uint64)
        self._engine._check(self._lib.mirsha_pipeline_trace(self._engine.ctx, self.handle, _ptr(out), n.value,
                                                            ctypes.byref(n)))
        return out

    def close(self) -> None:
        if getattr(self, "handle", None):
            self._lib.mirsha_pipeline_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CheckpointChains:
    """Streaming checkpoint chains on the device (mirsha_chains_*): one running
    SHA-256 per application node, as testengine's NodeState.ActiveHash
    (testengine/recorder.go:186-256).  write() = ActiveHash.Write of committed
    request digests, sum() = ActiveHash.Sum(nil) (state unchanged),
    reset() = NodeState.Set's fresh hasher."""

    def __init__(self, engine: Engine, n_chains: int):
        self._engine = engine
        self._lib = engine._lib
        h = ctypes.c_void_p()
        engine._check(self._lib.mirsha_chains_create(engine.ctx, int(n_chains), ctypes.byref(h)))
        self.handle = h
        self.n = int(n_chains)

    def write(self, digests, chain_of) -> None:
        d = np.ascontiguousarray(digests, dtype=np.uint8).reshape(-1, 32)
        c = np.ascontiguousarray(chain_of, dtype=np.uint32).reshape(-1)
        if c.size != d.shape[0]:
            raise ValueError("one chain id per digest")
        if c.size:
            self._engine._check(self._lib.mirsha_chains_absorb(self._engine.ctx, self.handle, _ptr(d), _ptr(c),
                                                               c.size))

    def sum(self, which) -> np.ndarray:
        w = np.ascontiguousarray(which, dtype=np.uint32).reshape(-1)
        out = np.empty((w.size, 32), dtype=np.uint8)
        if w.size:
            self._engine._check(self._lib.mirsha_chains_sum(self._engine.ctx, self.handle, _ptr(w), w.size,
                                                            _ptr(out)))
        return out

    def reset(self, which) -> None:
        w = np.ascontiguousarray(which, dtype=np.uint32).reshape(-1)
        if w.size:
            self._engine._check(self._lib.mirsha_chains_reset(self._engine.ctx, self.handle, _ptr(w), w.size))

    def close(self) -> None:
        if getattr(self, "handle", None):
            self._lib.mirsha_chains_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def bucket_order(length: Sequence[int]) -> tuple[np.ndarray, bool]:
    """Message order sorted by block count, longest first (stable); (order, is_identity)."""
    ln = np.ascontiguousarray(length, dtype=np.uint32)
    order = np.empty(ln.size, dtype=np.uint32)
    rc = _lib.load().mirsha_bucket_order(_ptr(ln), ln.size, _ptr(order))
    if rc < 0:
        raise MirshaError(rc, "bucket_order")
    return order, bool(rc == 1)


def hash_batch_multi(devices: Iterable[int], arena, off, length) -> np.ndarray:
    """Request-range sharding over several devices in one process; host gather."""
    devs = np.ascontiguousarray(list(devices), dtype=np.int32)
    a = _as_u8(arena)
    o = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(length, dtype=np.uint32)
    out = np.empty((o.size, 32), dtype=np.uint8)
    rc = _lib.load().mirsha_hash_batch_multi(_ptr(devs), devs.size, _ptr(a), a.size, _ptr(o), _ptr(ln), o.size, _ptr(out))
    check(rc)
    return out


class MultiEngine:
    """The multi-GPU drop-in (mirsha_multi, include/mirsha.h): one context
    per listed device, requests cut into contiguous ranges of equal bytes,
    each range packed, copied over its device's own PCIe link and hashed in
    parallel; digests in origin order.  A device may be listed twice (two
    contexts on one GPU: tests on a one-GPU box)."""

    def __init__(self, devices: Iterable[int]):
        self._lib = _lib.load()
        devs = np.ascontiguousarray(list(devices), dtype=np.int32)
        h = ctypes.c_void_p()
        check(self._lib.mirsha_multi_create(_ptr(devs), int(devs.size), ctypes.byref(h)))
        self.handle = h
        self.devices = [int(d) for d in devs]
        self._outstanding = {}

    def _check(self, rc: int) -> None:
        if rc != _lib.MIRSHA_OK:
            raw = self._lib.mirsha_multi_last_error(self.handle)
            raise MirshaError(rc, raw.decode() if raw else "")

    def context(self, k: int):
        """The ctypes handle of device index k's context (owned by this object)."""
        return self._lib.mirsha_multi_ctx(self.handle, int(k))

    def set_variant(self, variant: int) -> None:
        for k in range(len(self.devices)):
            check(self._lib.mirsha_ctx_set_variant(self.context(k), int(variant)))

    def hash_slice_arrays(self, sl: "SliceArrays") -> np.ndarray:
        out = np.empty((sl.n, 32), dtype=np.uint8)
        if sl.n:
            self._check(self._lib.mirsha_hash_slices_multi(self.handle, sl.ptr_p, sl.len_p, sl.first_p, sl.n,
                                                           _ptr(out)))
        return out

    def hash_slices(self, requests) -> np.ndarray:
        sl = requests if isinstance(requests, SliceArrays) else SliceArrays.from_requests(requests)
        return self.hash_slice_arrays(sl)

    def hash_arena(self, arena, off, length, out=None) -> np.ndarray:
        """mirsha_hash_arena_multi: requests packed in one arena (offsets, lengths)."""
        a = _as_u8(arena)
        o = np.ascontiguousarray(off, dtype=np.uint64)
        ln = np.ascontiguousarray(length, dtype=np.uint32)
        out = _out_rows(out, o.size)
        if o.size:
            self._check(self._lib.mirsha_hash_arena_multi(self.handle, _ptr(a), a.size, _ptr(o), _ptr(ln), o.size,
                                                          _ptr(out)))
        return out

    def host_empty(self, nbytes: int) -> np.ndarray:
        """Page-locked host memory usable by every device (mirsha_multi_host_alloc)."""
        p = ctypes.c_void_p()
        self._check(self._lib.mirsha_multi_host_alloc(self.handle, int(nbytes), ctypes.byref(p)))
        buf = (ctypes.c_uint8 * max(int(nbytes), 1)).from_address(p.value)
        arr = np.frombuffer(buf, dtype=np.uint8, count=int(nbytes))
        import weakref

        weakref.finalize(buf, self._lib.mirsha_host_free, p.value)
        return arr

    def submit_slices(self, requests, dedup: bool = False) -> "Ticket":
        sl = requests if isinstance(requests, SliceArrays) else SliceArrays.from_requests(requests)
        out = np.empty((sl.n, 32), dtype=np.uint8)
        t = ctypes.c_uint64(0)
        self._check(self._lib.mirsha_submit_slices_multi(self.handle, sl.ptr_p, sl.len_p, sl.first_p, sl.n,
                                                         _ptr(out), _lib.MIRSHA_SUBMIT_DEDUP if dedup else 0,
                                                         ctypes.byref(t)))
        self._outstanding[t.value] = out
        for k in [k for k in self._outstanding if k <= t.value - ASYNC_SLOTS]:
            del self._outstanding[k]
        return Ticket(t.value, out)

    def submit_arena(self, arena, off, length, out=None) -> "Ticket":
        """mirsha_submit_arena_multi: Engine.submit_batch over every device."""
        a = _as_u8(arena)
        o = np.ascontiguousarray(off, dtype=np.uint64)
        ln = np.ascontiguousarray(length, dtype=np.uint32)
        if o.shape != ln.shape:
            raise ValueError("off and len differ in length")
        n = int(o.size)
        out = _out_rows(out, n)
        t = ctypes.c_uint64(0)
        self._check(self._lib.mirsha_submit_arena_multi(self.handle, _ptr(a), a.size, _ptr(o), _ptr(ln), n, _ptr(out),
                                                        ctypes.byref(t)))
        self._outstanding[t.value] = (out, a)
        for k in [k for k in self._outstanding if k <= t.value - ASYNC_SLOTS]:
            del self._outstanding[k]
        return Ticket(t.value, out)

    def wait(self, ticket: "Ticket") -> np.ndarray:
        self._check(self._lib.mirsha_wait_multi(self.handle, ticket.value))
        for k in [k for k in self._outstanding if k <= ticket.value]:
            del self._outstanding[k]
        return ticket.out

    def poll(self, ticket: "Ticket") -> bool:
        done = ctypes.c_int(0)
        self._check(self._lib.mirsha_poll_multi(self.handle, ticket.value, ctypes.byref(done)))
        return bool(done.value)

    def last_cut(self) -> list:
        """First request of each device index in the last call, then n."""
        buf = (ctypes.c_uint32 * (len(self.devices) + 1))()
        n = self._lib.mirsha_multi_last_cut(self.handle, buf, len(buf))
        return list(buf)[:n]

    def host_profile(self, k: int) -> dict:
        buf = (ctypes.c_double * len(Engine.HOST_PHASES))()
        n = self._lib.mirsha_multi_host_profile(self.handle, int(k), buf, len(Engine.HOST_PHASES))
        if n < 0:
            self._check(n)
        return {key: buf[i] for i, key in enumerate(Engine.HOST_PHASES)}

    def close(self) -> None:
        if getattr(self, "handle", None):
            self._lib.mirsha_multi_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


__all__ = [
    "Engine",
    "MultiEngine",
    "CheckpointChains",
    "SliceArrays",
    "Ticket",
    "dedup_plan",
    "Pipeline",
    "bucket_order",
    "device_count",
    "hash_batch_multi",
    "MIRSHA_NULL_INDEX",
    "KERNEL_MSGS",
    "KERNEL_LISTS",
    "KERNEL_GEN",
    "KERNEL_CHAIN",
    "KERNEL_FUSED",
    "KERNEL_OVERLAP",
    "PIPELINE_SEQUENTIAL",
    "PIPELINE_FUSED",
    "PIPELINE_AUTO",
    "VARIANT_LDS",
    "VARIANT_DIRECT",
    "VARIANT_LOWOCC",
    "VARIANT_LDS_ONLY",
    "VARIANT_CU",
    "VARIANT_PAIR",
    "VARIANTS",
]
