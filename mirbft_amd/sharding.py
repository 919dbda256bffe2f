"""Request-range sharding across GPUs.

Independent hash requests (actions.go:22-23) shard by contiguous request range;
cuts fall on batch boundaries so each GPU's dependent batch-digest pass reads
only its own device-resident request digests.  No collective: a host gather
(concatenation in rank order) restores origin order.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np


def blocks_for_len(length) -> np.ndarray:
    """SHA-256 compressions per message: ceil((L + 9) / 64)."""
    return (np.asarray(length, dtype=np.uint64) + 72) >> 6


def shard_ranges(n_req: int, world: int, batch_size: int = 1,
                 lengths: Optional[Sequence[int]] = None) -> list[tuple[int, int]]:
    """[lo, hi) request range per rank, cut on multiples of ``batch_size``.

    With ``lengths`` the cuts balance total compressions, else request counts.
    """
    if world <= 0:
        raise ValueError("world must be positive")
    if n_req <= 0:
        return [(0, 0)] * world
    bs = max(1, int(batch_size))
    n_units = (n_req + bs - 1) // bs
    if lengths is None:
        w = np.full(n_units, bs, dtype=np.float64)
        w[-1] = n_req - (n_units - 1) * bs
    else:
        blk = blocks_for_len(lengths).astype(np.float64)
        pad = n_units * bs - n_req
        if pad:
            blk = np.concatenate([blk, np.zeros(pad)])
        w = blk.reshape(n_units, bs).sum(axis=1)
    cum = np.cumsum(w)
    total = cum[-1]
    cuts = [0]
    for r in range(1, world):
        u = int(np.searchsorted(cum, total * r / world, side="left")) + 1
        u = min(max(u, cuts[-1]), n_units)
        cuts.append(u)
    cuts.append(n_units)
    return [(min(a * bs, n_req), min(b * bs, n_req)) for a, b in zip(cuts[:-1], cuts[1:])]


def batch_lists(n_req: int, batch_size: int, first_req: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """(idx, batch_first) for consecutive BatchSize groups of request digests,
    in origin order (the last batch may be short).  idx is relative to first_req."""
    n_b = (n_req + batch_size - 1) // batch_size
    idx = np.arange(n_req, dtype=np.uint32)
    first = np.minimum(np.arange(n_b + 1, dtype=np.int64) * batch_size, n_req).astype(np.uint32)
    return idx, first


# One device launch addresses at most MIRSHA_MAX_DEVICE_ARENA_BYTES of arena
# (32-bit buffer offsets, include/mirsha.h); larger device-resident streams
# (BASELINE config 5: ~123 GB of mixed-size requests per GPU) are hashed in
# contiguous origin-order windows, each with its own length-bucketed order.
MAX_WINDOW_BYTES = 0xFFFFFF00


def arena_windows(off, length, max_bytes: int = MAX_WINDOW_BYTES) -> list[tuple[int, int, int]]:
    """Split requests (origin order, ascending offsets) into windows [i0, i1)
    whose bytes [off[i0], off[i1-1] + len[i1-1]) span at most max_bytes.
    Returns (i0, i1, base) with base = off[i0]."""
    off = np.asarray(off, dtype=np.uint64)
    ln = np.asarray(length, dtype=np.uint64)
    n = off.size
    if n == 0:
        return []
    end = off + ln
    if np.any(ln > max_bytes):
        raise ValueError("a single message exceeds the window size")
    out = []
    i0 = 0
    while i0 < n:
        base = int(off[i0])
        # last request whose end fits in [base, base + max_bytes]
        i1 = int(np.searchsorted(end, base + max_bytes, side="right"))
        i1 = max(i1, i0 + 1)
        out.append((i0, i1, base))
        i0 = i1
    return out


def window_orders(length, windows) -> np.ndarray:
    """Concatenated per-window processing orders (indices relative to the
    window start), each longest-first by block count, stable (mirsha_bucket_order)."""
    blk = blocks_for_len(length).astype(np.int64)
    parts = [np.argsort(-blk[i0:i1], kind="stable").astype(np.uint32) for i0, i1, _ in windows]
    return np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint32)
