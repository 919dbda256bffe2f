"""ctypes wrapper of the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")
NULL = 0xFFFFFFFF

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


class _BuildLock:
    """An exclusive flock on oracle/.build.lock around the staleness check, the
    rebuild and the dlopen: bench.py's ranks all self-check at once, and one
    must never dlopen a library another is still writing.  No lock (and no
    rebuild race to guard) when the directory is read-only."""

    def __enter__(self):
        import fcntl

        try:
            self.f = open(os.path.join(ORACLE_DIR, ".build.lock"), "w")
        except OSError:
            self.f = None
            return self
        fcntl.flock(self.f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        if self.f is not None:
            self.f.close()  # releases the flock


def _load_fresh(so: str, src: str) -> ctypes.CDLL:
    with _BuildLock():
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
            build()
        return ctypes.CDLL(so)


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    lib = _load_fresh(ORACLE_SO, os.path.join(ORACLE_DIR, "sha256_oracle.c"))
    vp = ctypes.c_void_p
    lib.oracle_hash_requests.argtypes = [vp, vp, vp, ctypes.c_uint32, vp]
    lib.oracle_hash_requests_mt.argtypes = [vp, vp, vp, ctypes.c_uint32, vp, ctypes.c_int]
    lib.oracle_hash_slices.argtypes = [vp, vp, vp, ctypes.c_uint32, vp]
    lib.oracle_batch_digests.argtypes = [vp, vp, vp, ctypes.c_uint32, vp]
    lib.oracle_gen_requests.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, vp]
    lib.oracle_sha256_force_impl.argtypes = [ctypes.c_int]
    lib.oracle_sha256_has_shani.restype = ctypes.c_int
    lib.oracle_mixed_data_len.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
    lib.oracle_mixed_data_len.restype = ctypes.c_uint32
    lib.oracle_gen_mixed.argtypes = [ctypes.c_uint64, vp, ctypes.c_uint64, vp, vp, vp]
    lib.oracle_mixed_lengths.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, vp]
    lib.oracle_splitmix64.argtypes = [ctypes.c_uint64]
    lib.oracle_splitmix64.restype = ctypes.c_uint64
    _lib = lib
    return lib


def _p(a: np.ndarray):
    return a.ctypes.data if a.size else None


def hash_requests(arena, off, length, threads: int = 1) -> np.ndarray:
    lib = load()
    a = np.ascontiguousarray(np.frombuffer(memoryview(arena), dtype=np.uint8) if not isinstance(arena, np.ndarray)
                             else arena.reshape(-1).view(np.uint8))
    o = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(length, dtype=np.uint32)
    out = np.empty((o.size, 32), dtype=np.uint8)
    if o.size:
        if threads > 1:
            lib.oracle_hash_requests_mt(_p(a), _p(o), _p(ln), o.size, _p(out), threads)
        else:
            lib.oracle_hash_requests(_p(a), _p(o), _p(ln), o.size, _p(out))
    return out


def hash_slices(slice_ptr: np.ndarray, slice_len: np.ndarray, first: np.ndarray, out: np.ndarray = None) -> np.ndarray:
    """processor.go:133-143 over HashRequest.Data slice lists (addresses as uint64)."""
    n = int(first.size) - 1
    if out is None:
        out = np.empty((n, 32), dtype=np.uint8)
    if n:
        load().oracle_hash_slices(_p(slice_ptr), _p(slice_len), _p(first), n, _p(out))
    return out


def hash_messages(messages) -> np.ndarray:
    lens = np.array([len(m) for m in messages], dtype=np.uint32)
    off = np.zeros(len(messages), dtype=np.uint64)
    if len(messages) > 1:
        np.cumsum(lens[:-1], out=off[1:])
    return hash_requests(b"".join(messages) or b"\0", off, lens)


def batch_digests(req_digests: np.ndarray, idx, first) -> np.ndarray:
    lib = load()
    d = np.ascontiguousarray(req_digests, dtype=np.uint8).reshape(-1, 32)
    ix = np.ascontiguousarray(idx, dtype=np.uint32)
    fs = np.ascontiguousarray(first, dtype=np.uint32)
    nb = fs.size - 1
    out = np.empty((nb, 32), dtype=np.uint8)
    if nb:
        lib.oracle_batch_digests(_p(d), _p(ix), _p(fs), nb, _p(out))
    return out


def gen_requests(seed: int, first: int, count: int, data_len: int) -> np.ndarray:
    lib = load()
    out = np.empty(count * (16 + data_len), dtype=np.uint8)
    lib.oracle_gen_requests(seed, first, count, data_len, _p(out))
    return out


def mixed_data_len(seed: int, i: int) -> int:
    """BASELINE config 5 data length of request i (oracle.h, oracle_mixed_data_len)."""
    return int(load().oracle_mixed_data_len(seed, i))


def mixed_lengths(seed: int, first: int, count: int) -> np.ndarray:
    """Request lengths (header + data) of config-5 requests [first, first + count)."""
    out = np.empty(count, dtype=np.uint32)
    if count:
        load().oracle_mixed_lengths(seed, first, count, _p(out))
    return out


def gen_mixed(seed: int, ids) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Config-5 messages of the request ids (any order), packed densely: (arena, off, len)."""
    lib = load()
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    total = int(sum(16 + lib.oracle_mixed_data_len(seed, int(i)) for i in ids))
    arena = np.empty(max(total, 1), dtype=np.uint8)
    off = np.empty(ids.size, dtype=np.uint64)
    ln = np.empty(ids.size, dtype=np.uint32)
    if ids.size:
        lib.oracle_gen_mixed(seed, _p(ids), ids.size, _p(arena), _p(off), _p(ln))
    return arena[:total], off, ln


EVP_SO = os.path.join(ORACLE_DIR, "libevp_loop.so")
_evp = None


def load_evp() -> ctypes.CDLL:
    """oracle/libevp_loop.so: the reference loop through OpenSSL's EVP SHA-256
    (BASELINE.md's "OpenSSL stand-in for Go crypto/sha256")."""
    global _evp
    if _evp is not None:
        return _evp
    lib = _load_fresh(EVP_SO, os.path.join(ORACLE_DIR, "evp_loop.c"))
    vp = ctypes.c_void_p
    lib.evp_hash_requests.argtypes = [vp, vp, vp, ctypes.c_uint32, vp, ctypes.c_int, ctypes.c_int]
    lib.evp_batch_digests.argtypes = [vp, vp, vp, ctypes.c_uint32, vp]
    lib.evp_version.restype = ctypes.c_char_p
    _evp = lib
    return lib


def evp_hash_requests(arena, off, length, threads: int = 1, split: bool = True) -> np.ndarray:
    """processor.go:133-143 through EVP (three Writes per request when split)."""
    lib = load_evp()
    a = np.ascontiguousarray(np.asarray(arena).reshape(-1).view(np.uint8))
    o = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(length, dtype=np.uint32)
    out = np.empty((o.size, 32), dtype=np.uint8)
    if o.size and lib.evp_hash_requests(_p(a), _p(o), _p(ln), o.size, _p(out), int(threads), int(split)):
        raise RuntimeError("evp_hash_requests failed")
    return out


def evp_batch_digests(req_digests: np.ndarray, idx, first) -> np.ndarray:
    lib = load_evp()
    d = np.ascontiguousarray(req_digests, dtype=np.uint8).reshape(-1, 32)
    ix = np.ascontiguousarray(idx, dtype=np.uint32)
    fs = np.ascontiguousarray(first, dtype=np.uint32)
    nb = fs.size - 1
    out = np.empty((nb, 32), dtype=np.uint8)
    if nb and lib.evp_batch_digests(_p(d), _p(ix), _p(fs), nb, _p(out)):
        raise RuntimeError("evp_batch_digests failed")
    return out


def evp_version() -> str:
    return load_evp().evp_version().decode()


def force_impl(impl: int) -> None:
    load().oracle_sha256_force_impl(impl)


def has_shani() -> bool:
    return bool(load().oracle_sha256_has_shani())
