#!/usr/bin/env python3
"""One traced fused config-3 run (GPU box): per tile queue, how many tiles,
which wave slots served them, and their end-time quantiles (us from the
first tile start); the list chunks' readiness-pass times.  Compare builds
with MIRSHA_AB_LIB.  Usage: trace_queues.py [requests]"""
import os

os.environ["MIRSHA_AB"] = "1"
os.environ["MIRSHA_FUSED_TRACE"] = "1"
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mirbft_amd import Engine, sharding  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18  # requests (64 per tile)
    data_len, bs = 4096, 500
    stride = 16 + data_len
    d_arena = torch.empty(n * stride, dtype=torch.uint8, device=dev)
    eng.synth_requests_device(0x6D69726266740003, 0, n, data_len, d_arena.data_ptr())
    d_off = torch.arange(n, dtype=torch.int64, device=dev) * stride
    d_len = torch.full((n,), stride, dtype=torch.int32, device=dev)
    d_req = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    idx, first = sharding.batch_lists(n, bs)
    d_bat = torch.empty((first.size - 1, 32), dtype=torch.uint8, device=dev)
    plan = eng.pipeline(n, idx, first, np.full(n, stride), mode="fused")
    for _ in range(30):
        eng.hash_requests_then_batches_device(plan, d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(),
                                              d_len.data_ptr(), d_req.data_ptr(), d_bat.data_ptr())
    plan.status()
    tr = plan.trace().astype(np.int64)
    nt, nc, ng = plan.shape()
    t = tr[: 3 * nt].reshape(nt, 3)
    ok = t[:, 0] > 0
    t0 = t[ok, 0].min()
    start, end, info = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0, t[:, 2]
    q = (info >> 40) & 0xF
    slot = (info >> 44) & 0xF
    for qq in sorted(set(q[ok].tolist())):
        m = ok & (q == qq)
        e = np.sort(end[m])
        print(f"queue {qq}: {m.sum()} tiles, slots {sorted(set(slot[m].tolist()))}, start med {np.median(start[m]):.0f}"
              f" us, end p10/50/90/max {e[len(e)//10]:.0f}/{e[len(e)//2]:.0f}/{e[9*len(e)//10]:.0f}/{e[-1]:.0f} us")
    print("untraced tiles (split tiles' segments):", int((~ok).sum()))
    isimd = (info >> 48) & 0xF
    psimd = (info >> 4) & 3
    lb = (info >> 52) & 1
    hwave = info & 15
    for qq in sorted(set(q[ok].tolist())):
        m = ok & (q == qq)
        print(f"queue {qq}: hw wave ids {np.bincount(hwave[m], minlength=16)[:8].tolist()}, identity != physical SIMD "
              f"{int((isimd[m] != psimd[m]).sum())}, in list blocks {int(lb[m].sum())}")
    for qq in (0, 1):
        m = np.flatnonzero(ok & (q == qq))
        late = m[np.argsort(end[m])[-6:]]
        for i in late:
            hw = int(info[i]) & 0xFFFFFFFF
            print(f"  late q{qq} tile {i}: start {start[i]:.0f} end {end[i]:.0f} us, hw simd {(hw >> 4) & 3} wave "
                  f"{hw & 15} cu {(hw >> 8) & 15} sh {(hw >> 12) & 1} se {(hw >> 13) & 7} xcc {(int(info[i]) >> 32) & 0xFF}"
                  f" slot {int(slot[i])} identity simd {int(isimd[i])} list block {int(lb[i])}")
    lone = ok & (info < 0)  # bit 63: the tile ran blocks as its SIMD's only live wave (from bit 53..62's block)
    if lone.any():
        lb0 = (info >> 53) & 0x3FF
        print(f"lone-wave tiles: {int(lone.sum())}, first lone block p10/50/90 "
              f"{np.percentile(lb0[lone], [10, 50, 90]).tolist()}")
        # per physical SIMD: the lone stretch starts when the SIMD's other tile
        # waves end (their tiles' ends), so a lone tile's block time is
        # (its end - that) / (blocks left after its first lone block)
        hwv = info & 0xFFFFFFFF
        loc = ((info >> 32) & 0xFF) * 4096 + ((hwv >> 13) & 7) * 512 + ((hwv >> 12) & 1) * 256 + ((hwv >> 8) & 15) * 16 \
            + ((hwv >> 4) & 3)
        other_end = {}
        for i in np.flatnonzero(ok & ~lone):
            other_end[int(loc[i])] = max(other_end.get(int(loc[i]), 0.0), float(end[i]))
        rates = []
        for i in np.flatnonzero(lone):
            t_alone = other_end.get(int(loc[i]))
            left = 65 - int(lb0[i])
            if t_alone is not None and left >= 8 and end[i] > t_alone:
                rates.append((end[i] - t_alone) / left)
        if rates:
            print(f"lone stretch us per block (config-3 tiles, >= 8 blocks left): n {len(rates)}, p10/50/90 "
                  f"{np.round(np.percentile(rates, [10, 50, 90]), 2).tolist()}")
    else:
        print("lone-wave tiles: none")
    passed = (tr[3 * nt: 3 * nt + nc] - t0) / 100.0
    print("readiness chunks passed p10/50/90/max us:", [round(float(np.percentile(passed, p)), 0) for p in (10, 50, 90, 100)])
    gend = (tr[3 * nt + nc: 3 * nt + nc + ng] - t0) / 100.0
    print("list groups end us:", [round(float(x)) for x in gend])


if __name__ == "__main__":
    main()
