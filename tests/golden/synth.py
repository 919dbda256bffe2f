"""Deterministic synthetic inputs shared by the fixture generator and the tests.

splitmix64 (vectorised with numpy uint64 wrap-around) — the same stream as
oracle_gen_requests (oracle/sha256_oracle.c) and the device generator
(mirbft_amd/csrc/mirsha_kernels.hip gen_requests_kernel).
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 0x6D69726266740000  # "mirbft\0\0" (SURVEY.md §8d); seed = SEED_BASE + config_id

_G = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def data_bytes(seed: int, i: int, n: int) -> bytes:
    """n bytes: 8-byte word j = splitmix64(splitmix64(seed ^ i) + j), little endian."""
    key = splitmix64(np.uint64((seed ^ i) & 0xFFFFFFFFFFFFFFFF))
    with np.errstate(over="ignore"):
        words = splitmix64(key + np.arange((n + 7) // 8, dtype=np.uint64))
    return words.astype("<u8").tobytes()[:n]


def request_message(seed: int, i: int, data_len: int) -> bytes:
    """Synthetic request i: LE64(i % 16) || LE64(i // 16) || data (state_machine.go:313-317 layout)."""
    return (i % 16).to_bytes(8, "little") + (i // 16).to_bytes(8, "little") + data_bytes(seed, i, data_len)


def request_arena(seed: int, first: int, count: int, data_len: int) -> np.ndarray:
    """Densely packed messages [first, first+count) — vectorised request_message."""
    stride = 16 + data_len
    out = np.zeros((count, stride), dtype=np.uint8)
    idx = np.arange(first, first + count, dtype=np.uint64)
    out[:, 0:8] = (idx % np.uint64(16)).astype("<u8").view(np.uint8).reshape(count, 8)
    out[:, 8:16] = (idx // np.uint64(16)).astype("<u8").view(np.uint8).reshape(count, 8)
    nw = (data_len + 7) // 8
    if nw:
        key = splitmix64(np.uint64(seed) ^ idx)
        with np.errstate(over="ignore"):
            words = splitmix64(key[:, None] + np.arange(nw, dtype=np.uint64)[None, :])
        out[:, 16:] = words.astype("<u8").view(np.uint8).reshape(count, nw * 8)[:, :data_len]
    return out.reshape(-1)


def pattern_bytes(n: int, salt: int = 0) -> bytes:
    """Cheap deterministic byte pattern for boundary-length vectors."""
    return bytes(((j * 131 + n * 7 + salt) & 0xFF) for j in range(n))


def log_uniform_lengths(seed: int, count: int, lo_log2: int = 6, hi_log2: int = 16) -> np.ndarray:
    """Integer log-uniform-by-octave lengths in [2^lo, 2^hi): octave k uniform in
    [lo, hi), then uniform inside the octave.  Integer-only, so host and device agree."""
    r = splitmix64(np.uint64(seed) ^ np.arange(count, dtype=np.uint64))
    k = (r % np.uint64(hi_log2 - lo_log2)).astype(np.int64) + lo_log2
    base = np.left_shift(np.int64(1), k)
    m = ((r >> np.uint64(8)) % base.astype(np.uint64)).astype(np.int64)
    return (base + m).astype(np.uint32)
