#!/usr/bin/env python3
"""Timeline of config 3's overlapped launch (GPU box): per-tile start / end
stamps of the fused plan's tile waves with the previous cycle's chains (steady
state) and without them (tiles only), and how the SIMDs finish.  Usage:
trace_overlap.py [reps]"""
import json
import os

os.environ["MIRSHA_AB"] = "1"  # the library reads the trace knob only with MIRSHA_AB=1
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mirbft_amd import Engine, sharding  # noqa: E402


def pcts(a):
    return [round(float(np.percentile(a, p)), 1) for p in (0, 1, 10, 50, 90, 99, 100)]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = torch.cuda.Stream(dev)
    eng = Engine(0)
    eng.set_stream(s.cuda_stream)
    n, data_len, bs = 1 << 18, 4096, 500
    stride = 16 + data_len
    d_arena = torch.empty(n * stride, dtype=torch.uint8, device=dev)
    eng.synth_requests_device(0x6D69726266740003, 0, n, data_len, d_arena.data_ptr())
    d_off = torch.arange(n, dtype=torch.int64, device=dev) * stride
    d_len = torch.full((n,), stride, dtype=torch.int32, device=dev)
    d_req = [torch.empty((n, 32), dtype=torch.uint8, device=dev) for _ in range(2)]
    idx, first = sharding.batch_lists(n, bs)
    d_bat = torch.empty((first.size - 1, 32), dtype=torch.uint8, device=dev)
    os.environ["MIRSHA_FUSED_TRACE"] = "1"
    plan = eng.pipeline(n, idx, first, np.full(n, stride), mode="fused")
    os.environ.pop("MIRSHA_FUSED_TRACE", None)
    args = (d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(), d_len.data_ptr())
    nt, nc, ng = plan.shape()
    for form, prev in (("chains", d_req[1].data_ptr()), ("tiles_only", 0)):
        for _ in range(reps):
            eng.pipeline_overlap_device(plan, *args, d_req[0].data_ptr(), prev, d_bat.data_ptr())
        eng.sync()
        plan.status()
        tr = plan.trace().astype(np.int64)
        ts, te, info = tr[0:3 * nt:3], tr[1:3 * nt:3], tr[2:3 * nt:3]
        traced = ts > 0  # split tiles run as segments and carry no tile stamps
        ts, te, info = ts[traced], te[traced], info[traced]
        hw = info & 0xFFFFFFFF
        xcc = (info >> 32) & 0xFF
        simd_key = xcc << 20 | ((hw >> 8) & 0xFF) << 4 | (hw >> 4) & 0x3  # XCC, SE / SH / CU, SIMD
        slot = (info >> 44) & 0xF
        gend = tr[3 * nt + nc:3 * nt + nc + ng]
        t0 = ts.min()
        us = lambda x: (x - t0) / 100.0  # noqa: E731  (100 MHz ticks -> us)
        keys, inv = np.unique(simd_key, return_inverse=True)
        simd_end = np.zeros(keys.size)
        simd_tiles = np.zeros(keys.size, dtype=np.int64)
        np.maximum.at(simd_end, inv, us(te))
        np.add.at(simd_tiles, inv, 1)
        # active tile waves over time (10 us bins)
        span = float(us(te.max()))
        bins = np.arange(0.0, span + 10.0, 10.0)
        active = [int(((us(ts) <= b) & (us(te) > b)).sum()) for b in bins]
        res = {"form": form, "tiles_traced": int(traced.sum()), "tiles": nt, "simds": int(keys.size),
               "span_us": round(span, 1), "tile_end_us": pcts(us(te)), "tile_start_us": pcts(us(ts)),
               "tile_dur_us": pcts((te - ts) / 100.0), "simd_end_us": pcts(simd_end),
               "simd_tiles": {int(k): int(v) for k, v in zip(*np.unique(simd_tiles, return_counts=True))},
               "simd_end_by_tiles": {int(k): pcts(simd_end[simd_tiles == k]) for k in np.unique(simd_tiles)},
               "slot_end_us": {int(k): pcts(us(te[slot == k])) for k in np.unique(slot)},
               "simd_end_by_xcc": {int(x): pcts(simd_end[(keys >> 20) == x]) for x in np.unique(keys >> 20)},
               "tile_start_by_xcc": {int(x): pcts(us(ts[xcc == x])) for x in np.unique(xcc)},
               "active_waves_10us": active,
               "group_end_us": pcts(us(gend[gend > 0])) if form == "chains" and (gend > 0).any() else None}
        print(json.dumps(res), flush=True)
    plan.close()
    eng.close()


if __name__ == "__main__":
    main()
