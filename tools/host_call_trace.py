#!/usr/bin/env python3
"""Host-API timeline of a config-2 call (2^20 x 272 B requests + BatchSize-20
batches) through mirsha_hash_requests_then_batches: per-call wall time, the
library's host phases, and (MIRSHA_STAGE_TRACE=1, stderr) the per-chunk queue /
wait / copy-out times of the pipelined path.  Pageable and pinned arenas.

Usage (GPU box):  MIRSHA_AB=1 MIRSHA_STAGE_TRACE=1 python tools/host_call_trace.py [reps]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import synth  # noqa: E402
from mirbft_amd import Engine, sharding  # noqa: E402


def main(reps):
    eng = Engine(0)
    n, stride = 1 << 20, 272
    arena = synth.request_arena(synth.SEED_BASE + 2, 0, n, 256)
    off = np.arange(n, dtype=np.uint64) * stride
    ln = np.full(n, stride, np.uint32)
    idx, first = sharding.batch_lists(n, 20)
    req = np.empty((n, 32), np.uint8)
    bat = np.empty((first.size - 1, 32), np.uint8)
    pinned = eng.host_empty(arena.size)
    pinned[:] = arena
    out = {}
    for name, src in (("pageable", arena), ("pinned", pinned)):
        eng.hash_requests_then_batches(src, off, ln, idx, first, out=req, batch_out=bat)  # warm
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            eng.hash_requests_then_batches(src, off, ln, idx, first, out=req, batch_out=bat)
            t.append((time.perf_counter() - t0) * 1e3)
            print(f"{name} call {t[-1]:.3f} ms {json.dumps(eng.host_profile())}", file=sys.stderr, flush=True)
        out[name] = {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
                     "gb_per_s_median": (n * stride + 32 * n) / np.median(t) / 1e6}
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 5)
