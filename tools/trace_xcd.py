#!/usr/bin/env python3
"""Per-XCD end times of the fused config-3 launch's last-queue tiles over
consecutive runs (GPU box): is the last queue's spread a stable per-XCD
property?  Usage: trace_xcd.py [runs]"""
import json
import os

os.environ["MIRSHA_AB"] = "1"  # trace knob
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mirbft_amd import Engine, sharding  # noqa: E402


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = torch.cuda.Stream(dev)
    eng = Engine(0)
    eng.set_stream(s.cuda_stream)
    data_len, n, bs = 4096, 1 << 18, 500
    stride = 16 + data_len
    d_arena = torch.empty(n * stride, dtype=torch.uint8, device=dev)
    eng.synth_requests_device(0x6D69726266740003, 0, n, data_len, d_arena.data_ptr())
    d_off = torch.arange(n, dtype=torch.int64, device=dev) * stride
    d_len = torch.full((n,), stride, dtype=torch.int32, device=dev)
    d_req = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    idx, first = sharding.batch_lists(n, bs)
    d_bat = torch.empty((first.size - 1, 32), dtype=torch.uint8, device=dev)
    os.environ["MIRSHA_FUSED_TRACE"] = "1"
    plan = eng.pipeline(n, idx, first, np.full(n, stride), mode="fused")
    os.environ.pop("MIRSHA_FUSED_TRACE", None)
    nt, nc, ng = plan.shape()

    def run():
        eng.hash_requests_then_batches_device(plan, d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(),
                                              d_len.data_ptr(), d_req.data_ptr(), d_bat.data_ptr())

    for _ in range(10):
        run()
    for r in range(runs):
        run()
        plan.status()
        tr = plan.trace().astype(np.int64)
        ts, te, info = tr[0:3 * nt:3], tr[1:3 * nt:3], tr[2:3 * nt:3]
        gend = tr[3 * nt + nc:3 * nt + nc + ng]
        ok = ts > 0
        ts, te, info, tid = ts[ok], te[ok], info[ok], np.nonzero(ok)[0]
        xcc, queue = (info >> 32) & 0xFF, (info >> 40) & 0xF
        t0 = ts.min()
        m3 = queue == 3
        per = {}
        for x in range(8):
            m = m3 & (xcc == x)
            if m.any():
                e = (te[m] - t0) / 100.0
                per[x] = [int(m.sum()), round(float(np.median(e)), 1), round(float(e.min()), 1), round(float(e.max()), 1)]
        # q3 tile index (needed-at order) vs end: rank correlation
        e3 = (te[m3] - t0) / 100.0
        rc = float(np.corrcoef(np.argsort(np.argsort(tid[m3])), np.argsort(np.argsort(e3)))[0, 1])
        print(json.dumps({"run": r, "q3_end_by_xcc": per, "q3_rank_corr_tile_vs_end": round(rc, 3),
                          "chains_end": round(float((gend.max() - t0) / 100.0), 1)}), flush=True)
    plan.close()
    eng.close()


if __name__ == "__main__":
    main()
