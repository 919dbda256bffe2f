#!/usr/bin/env python3
"""Config-3 launch forms, same box (GPU): the fused plan's overlapped launch
with chains (steady state) and without (a stream's first cycle: tiles only),
and the CU-block request kernel alone.  Kernel time by HIP events.
Usage: exp_overlap.py [reps] [overlap tile priority modes: balance progress queue ...]
(MIRSHA_FUSED_OVERLAP_PRIO, read with MIRSHA_AB=1 on every launch)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mirbft_amd import Engine, sharding  # noqa: E402
from mirbft_amd.engine import KERNEL_FUSED, KERNEL_MSGS  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    modes = sys.argv[2:] or [None]
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
    plan = eng.pipeline(n, idx, first, np.full(n, stride), mode="fused")
    args = (d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(), d_len.data_ptr())
    out = {"split_tiles": plan.split_tiles()}

    def timed(fn, timer):
        for _ in range(5):
            fn()
        eng.sync()
        eng.set_timing_mask([timer])
        eng.set_timing(True)
        eng.reset_timing()
        for _ in range(reps):
            fn()
        eng.sync()
        eng.set_timing(False)
        k, ms = eng.kernel_time(timer)
        return round(ms / max(k, 1) * 1e3, 1)

    for _ in range(2):
        for m in modes:
            sfx = f"_{m}" if m else ""
            if m:
                os.environ["MIRSHA_AB"] = "1"
                os.environ["MIRSHA_FUSED_OVERLAP_PRIO"] = m
            out.setdefault("overlap_chains_us" + sfx, []).append(timed(
                lambda: eng.pipeline_overlap_device(plan, *args, d_req[0].data_ptr(), d_req[1].data_ptr(),
                                                    d_bat.data_ptr()), KERNEL_FUSED))
            out.setdefault("overlap_tiles_only_us" + sfx, []).append(timed(
                lambda: eng.pipeline_overlap_device(plan, *args, d_req[0].data_ptr(), 0, d_bat.data_ptr()),
                KERNEL_FUSED))
            os.environ.pop("MIRSHA_FUSED_OVERLAP_PRIO", None)
        out.setdefault("fused_us", []).append(timed(
            lambda: eng.hash_requests_then_batches_device(plan, *args, d_req[0].data_ptr(), d_bat.data_ptr()),
            KERNEL_FUSED))
        out.setdefault("cu_kernel_us", []).append(timed(
            lambda: eng.hash_batch_device(*args, None, n, d_req[0].data_ptr()), KERNEL_MSGS))
    plan.status()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
