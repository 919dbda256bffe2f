#!/usr/bin/env python3
"""Per-tile timeline of the request kernel (diagnostic build, tools/ab_build.sh
stamps): runs BASELINE config 2 steps (request kernel + batch kernel, as
bench.py), then reads the last launch's stamps: per tile the 100 MHz time at
wave start, metadata ready, first block landed, end, plus the wave's HW_ID /
XCC_ID.  Writes <out>.npy (raw) and prints a JSON summary.

Usage (GPU box): MIRSHA_AB_LIB=tools/scratch/stamps/libmirsha.so python tools/stamp_run.py gpurun_out/x/stamps
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mirbft_amd import Engine, sharding  # noqa: E402
from mirbft_amd import _lib  # noqa: E402


def main(out):
    assert "stamps" in os.environ.get("MIRSHA_AB_LIB", ""), "needs a stamps build"
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    n, data_len, bs = 1 << 20, 256, 20
    stride = 16 + data_len
    d_arena = torch.empty(n * stride, dtype=torch.uint8, device=dev)
    d_off = torch.arange(n, dtype=torch.int64, device=dev) * stride
    d_len = torch.full((n,), stride, dtype=torch.int32, device=dev)
    d_req = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    idx, first = sharding.batch_lists(n, bs)
    d_bat = torch.empty((first.size - 1, 32), dtype=torch.uint8, device=dev)
    eng.synth_requests_device(0x6D69726266740002, 0, n, data_len, d_arena.data_ptr())
    plan = eng.pipeline(n, idx, first, np.full(n, stride))

    def step():
        eng.hash_requests_then_batches_device(plan, d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(),
                                              d_len.data_ptr(), d_req.data_ptr(), d_bat.data_ptr())

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for _ in range(8):
            step()
        torch.cuda.synchronize()
    step()
    torch.cuda.synchronize()
    lib = _lib.load()
    fn = lib.mirsha_ab_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    tiles = n // 64
    raw = np.zeros(6 * tiles, dtype=np.uint64)
    assert fn(raw.ctypes.data, raw.size) == 0
    raw = raw.reshape(tiles, 6)
    np.save(out + ".npy", raw)
    s = raw[:, :4].astype(np.int64)
    base = s[:, 0].min()
    rel = (s - base) / 100.0  # us
    hw, xcc = raw[:, 4].astype(np.int64), raw[:, 5].astype(np.int64)
    simd = (xcc << 16) | ((hw >> 4) & 0xFFF)  # simd/pipe/cu/sh/se bits + XCC
    span = rel[:, 3].max()
    summ = {
        "tiles": int(tiles), "span_us": float(span),
        "meta_us": np.percentile(rel[:, 1] - rel[:, 0], [10, 50, 90]).tolist(),
        "first_block_us": np.percentile(rel[:, 2] - rel[:, 1], [10, 50, 90]).tolist(),
        "compute_us": np.percentile(rel[:, 3] - rel[:, 2], [10, 50, 90]).tolist(),
        "wave_us": np.percentile(rel[:, 3] - rel[:, 0], [10, 50, 90]).tolist(),
        "start_us_pct": np.percentile(rel[:, 0], [0, 10, 25, 50, 75, 90, 100]).tolist(),
        "end_us_pct": np.percentile(rel[:, 3], [0, 10, 25, 50, 75, 90, 100]).tolist(),
        "simds": int(np.unique(simd).size),
    }
    # Per SIMD: resident waves over time (sweep), time with 0 resident waves,
    # and time where every resident wave is still before its first block.
    zero, prolog_only, avg = [], [], []
    for key in np.unique(simd):
        m = simd == key
        ev = []
        for a, b, c in zip(rel[m, 0], rel[m, 2], rel[m, 3]):
            ev += [(a, 1, 1), (b, 0, -1), (c, -1, 0)]  # (time, d_resident, d_waiting)
        ev.sort()
        res = wait = 0
        last = 0.0
        z = p = acc = 0.0
        for tt, dr, dw in ev:
            dt = tt - last
            if res == 0:
                z += dt
            elif wait == res:
                p += dt
            acc += res * dt
            res += dr
            wait += dw
            last = tt
        z += span - last
        zero.append(z / span)
        prolog_only.append(p / span)
        avg.append(acc / span)
    summ["simd_idle_frac"] = np.percentile(zero, [10, 50, 90]).tolist()
    summ["simd_all_waiting_frac"] = np.percentile(prolog_only, [10, 50, 90]).tolist()
    summ["simd_avg_waves"] = np.percentile(avg, [10, 50, 90]).tolist()
    print(json.dumps(summ))


if __name__ == "__main__":
    main(sys.argv[1])
