#!/usr/bin/env python3
"""Timeline of one fused run (GPU box): when tiles finish vs when list chunks
pass their readiness wait.  Usage: trace_fused.py <config> [pace ...]"""
import json
import os

os.environ["MIRSHA_AB"] = "1"  # the library reads the schedule / trace knobs only with MIRSHA_AB=1
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mirbft_amd import Engine, sharding  # noqa: E402


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    paces = [int(x) for x in sys.argv[2:]] or [0, 1]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = torch.cuda.Stream(dev)
    eng = Engine(0)
    eng.set_stream(s.cuda_stream)
    data_len, n, bs = {2: (256, 1 << 20, 20), 3: (4096, 1 << 18, 500)}[cfg]
    stride = 16 + data_len
    d_arena = torch.empty(n * stride, dtype=torch.uint8, device=dev)
    eng.synth_requests_device(0x6D69726266740000 + cfg, 0, n, data_len, d_arena.data_ptr())
    d_off = torch.arange(n, dtype=torch.int64, device=dev) * stride
    d_len = torch.full((n,), stride, dtype=torch.int32, device=dev)
    d_req = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    idx, first = sharding.batch_lists(n, bs)
    d_bat = torch.empty((first.size - 1, 32), dtype=torch.uint8, device=dev)
    for pace in paces:
        os.environ["MIRSHA_FUSED_TRACE"] = "1"
        if pace:
            os.environ["MIRSHA_FUSED_PACE"] = str(pace)
        plan = eng.pipeline(n, idx, first, np.full(n, stride), mode="fused")
        os.environ.pop("MIRSHA_FUSED_PACE", None)
        os.environ.pop("MIRSHA_FUSED_TRACE", None)
        for _ in range(20):
            eng.hash_requests_then_batches_device(plan, d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(),
                                                  d_len.data_ptr(), d_req.data_ptr(), d_bat.data_ptr())
        plan.status()
        tr = plan.trace().astype(np.int64)
        nt, nc, ng = plan.shape()
        ts, te, info = tr[0:3 * nt:3], tr[1:3 * nt:3], tr[2:3 * nt:3]
        chunk = tr[3 * nt:3 * nt + nc]
        gend = tr[3 * nt + nc:3 * nt + nc + ng]
        cend = tr[3 * nt + nc + ng:3 * nt + 2 * nc + ng]
        traced = ts > 0  # split tiles run as segments and carry no tile stamps
        ts, te, info = ts[traced], te[traced], info[traced]
        simd_key = ((info >> 32) & 0xFF) << 16 | ((info & 0xFFFFFFFF) >> 4) & 0xFFF
        queue, slot = (info >> 40) & 0xF, (info >> 44) & 0xF
        t0 = ts.min()
        us = lambda x: (x - t0) / 100.0  # noqa: E731  (100 MHz ticks -> us)
        dur = (te - ts) / 100.0
        q = lambda a: [round(float(np.percentile(a, p)), 1) for p in (0, 10, 50, 90, 100)]  # noqa: E731
        per_q = {}
        for qq in np.unique(queue):
            m = queue == qq
            per_q[int(qq)] = {"tiles": int(m.sum()), "end_us_pcts": q(us(te[m])), "dur_us_pcts": q(dur[m]),
                              "start_us_pcts": q(us(ts[m]))}
        # waves of one SIMD per queue (the slot assignment puts one of each queue on every SIMD)
        _, per_simd = np.unique(simd_key, return_counts=True)
        res = {"config": cfg, "pace": pace, "tiles": nt, "counters": nc, "groups": ng, "per_queue": per_q,
               "tiles_per_simd_pcts": q(per_simd),
               "tile_start_us_pcts": q(us(ts)), "tile_end_us_pcts": q(us(te)), "tile_dur_us_pcts": q(dur),
               "group_end_us": q(us(gend)), "kernel_span_us": round(float(us(max(te.max(), gend.max()))), 1)}
        # group 0's chunks: pass time vs when the tiles it needs ended (needed-at order rebuilt here)
        cpg = nc // max(ng, 1)
        res["group0_chunk_pass_us"] = [round(float(us(chunk[c])), 1) for c in range(0, min(cpg, 200), max(1, cpg // 16))]
        res["group0_chunk_compute_us"] = [round(float((cend[c] - chunk[c]) / 100.0), 1) for c in range(0, min(cpg, 40))]
        res["group0_chunk_gap_us"] = [round(float((chunk[c + 1] - cend[c]) / 100.0), 1) for c in range(0, min(cpg - 1, 40))]
        print(json.dumps(res), flush=True)
        plan.close()
    eng.close()


if __name__ == "__main__":
    main()
