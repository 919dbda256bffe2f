#!/usr/bin/env python3
"""Fused-pass experiments (GPU box): where does sha256_fused_kernel's time go?

  fused          config 2/3 plan, fused mode
  fused_nolists  same requests, no lists (request path cost inside the fused kernel)
  msgs           plain request kernel (identity order)
  msgs_posmajor  plain request kernel, fused plan's needed-at order
Prints one JSON line per case (kernel ms from HIP events on a private stream).
"""
import json
import os

os.environ["MIRSHA_AB"] = "1"  # the library reads the schedule / trace knobs only with MIRSHA_AB=1
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mirbft_amd import Engine, sharding  # noqa: E402


def timeit(s, fn, warm=30, reps=30):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = torch.cuda.Stream(dev)
    eng = Engine(0)
    eng.set_stream(s.cuda_stream)
    cfgs = [int(c) for c in (sys.argv[1:] or ["2", "3"])]
    for cfg in cfgs:
        data_len, n, bs = {2: (256, 1 << 20, 20), 3: (4096, 1 << 18, 500)}[cfg]
        stride = 16 + data_len
        d_arena = torch.empty(n * stride, dtype=torch.uint8, device=dev)
        eng.synth_requests_device(0x6D69726266740000 + cfg, 0, n, data_len, d_arena.data_ptr())
        d_off = torch.arange(n, dtype=torch.int64, device=dev) * stride
        d_len = torch.full((n,), stride, dtype=torch.int32, device=dev)
        d_req = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        idx, first = sharding.batch_lists(n, bs)
        d_bat = torch.empty((first.size - 1, 32), dtype=torch.uint8, device=dev)
        lens = np.full(n, stride)

        def run_plan(plan, nl):
            return lambda: eng.hash_requests_then_batches_device(plan, d_arena.data_ptr(), d_arena.numel(),
                                                                 d_off.data_ptr(), d_len.data_ptr(), d_req.data_ptr(),
                                                                 d_bat.data_ptr())

        out = {}
        plan = eng.pipeline(n, idx, first, lens, mode="fused")
        out["fused"] = timeit(s, run_plan(plan, first.size - 1))
        plan.status()
        want = (d_req.cpu().numpy().copy(), d_bat.cpu().numpy().copy())
        for pace in (1, 2, 3):
            os.environ["MIRSHA_FUSED_PACE"] = str(pace)
            pp = eng.pipeline(n, idx, first, lens, mode="fused")
            os.environ.pop("MIRSHA_FUSED_PACE")
            d_req.zero_()
            d_bat.zero_()
            out[f"paced{pace}"] = timeit(s, run_plan(pp, first.size - 1))
            pp.status()
            out[f"paced{pace}_ok"] = bool(np.array_equal(d_req.cpu().numpy(), want[0]) and
                                          np.array_equal(d_bat.cpu().numpy(), want[1]))
            pp.close()
        plan0 = eng.pipeline(n, np.zeros(0, np.uint32), np.zeros(1, np.uint32), lens, mode="fused")
        out["fused_nolists"] = timeit(s, run_plan(plan0, 0))
        plan0.status()
        out["msgs"] = timeit(s, lambda: eng.hash_batch_device(d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(),
                                                              d_len.data_ptr(), None, n, d_req.data_ptr()))
        # needed-at order = position within the batch (batch_lists is consecutive groups of bs)
        pos = np.arange(n) % bs
        order = np.argsort(pos, kind="stable").astype(np.int32)
        d_order = torch.from_numpy(order).to(dev)
        out["msgs_posmajor"] = timeit(s, lambda: eng.hash_batch_device(d_arena.data_ptr(), d_arena.numel(),
                                                                       d_off.data_ptr(), d_len.data_ptr(),
                                                                       d_order.data_ptr(), n, d_req.data_ptr()))
        print(json.dumps({"config": cfg, **{k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}}),
              flush=True)
        plan.close()
        plan0.close()
    eng.close()


if __name__ == "__main__":
    main()
