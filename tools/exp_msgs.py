#!/usr/bin/env python3
"""Request-kernel timing experiments (GPU box): how much of sha256_msgs_kernel's
time is memory placement vs VALU.  Prints one JSON line per case.

  normal      config 2 layout (2^20 x 272 B, packed)
  l2res       same lengths, offsets wrap every 8192 messages (2.2 MB: L2-resident)
  stride320   272-B messages at a 320-B (5-block) stride
  aligned256  256-B messages at 256-B stride
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mirbft_amd import Engine  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = Engine(0)
    s = torch.cuda.Stream(dev)  # non-null: the engine maps stream 0 to its own stream
    eng.set_stream(s.cuda_stream)
    n = 1 << 20
    arena = torch.randint(0, 256, (n * 320 + 64,), dtype=torch.uint8, device=dev)
    cases = {
        "normal": (272, 272, None),
        "l2res": (272, 272, 8192),
        "stride320": (272, 320, None),
        "aligned256": (256, 256, None),
        "len320": (320, 320, None),
    }
    which = sys.argv[1:] or list(cases)
    variants = [int(v) for v in os.environ.get("VARIANTS", "0").split(",")]
    for name in which:
        L, stride, wrap = cases[name]
        i = torch.arange(n, dtype=torch.int64, device=dev)
        if wrap:
            i = i % wrap
        d_off = i * stride
        d_len = torch.full((n,), L, dtype=torch.int32, device=dev)
        d_out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        for v in variants:
            eng.set_variant(v)

            def go():
                eng.hash_batch_device(arena.data_ptr(), arena.numel(), d_off.data_ptr(), d_len.data_ptr(), None, n,
                                      d_out.data_ptr())

            for _ in range(100):
                go()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 50
            e0.record(s)
            for _ in range(reps):
                go()
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            comps = n * ((L + 72) // 64)
            print(json.dumps({"case": name, "variant": v, "ms": ms, "gcomp_per_s": comps / ms / 1e6,
                              "frac_spec": comps * 1384 / (ms * 1e-3) / 78.6432e12}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
