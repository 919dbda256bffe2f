"""Timeline of the continuation plan (MIRSHA_PIPELINE_CONT) on BASELINE
config 2: when request tiles of each segment finish, when each (group,
segment) runs and how long it takes (s_memrealtime, 100 MHz).  GPU only:
python tools/cont_trace.py > gpurun_out/cont_trace.json"""
import json
import os
import sys

import numpy as np

os.environ["MIRSHA_CONT_TRACE"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from mirbft_amd import sharding  # noqa: E402
from mirbft_amd.engine import Engine  # noqa: E402


def main():
    n, data_len, bs = 1 << 20, 256, 20
    stride = 16 + data_len
    eng = Engine(0)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    d_arena = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    d_off = torch.arange(n, dtype=torch.int64, device="cuda") * stride
    d_len = torch.full((n,), stride, dtype=torch.int32, device="cuda")
    d_req = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    idx, first = sharding.batch_lists(n, bs)
    d_bat = torch.empty((first.size - 1, 32), dtype=torch.uint8, device="cuda")
    eng.synth_requests_device(0x6D69726266740002, 0, n, data_len, d_arena.data_ptr())
    plan = eng.pipeline(n, idx, first, np.full(n, stride), mode="cont")
    assert plan.mode_name == "cont"
    for _ in range(60):
        eng.hash_requests_then_batches_device(plan, d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(),
                                              d_len.data_ptr(), d_req.data_ptr(), d_bat.data_ptr())
    torch.cuda.synchronize()
    tr = plan.trace().astype(np.int64)
    bounds = plan.segments()
    S = len(bounds)
    n_tiles = (n + 63) // 64
    tiles = tr[: 2 * n_tiles].reshape(-1, 2)
    segs = tr[2 * n_tiles:].reshape(-1, S, 2)
    t0 = tiles[:, 0].min()
    us = lambda x: (np.asarray(x) - t0) / 100.0  # noqa: E731
    # segment of each tile position (processing order: segment-major)
    ords = np.arange(n) % bs
    seg_of = np.searchsorted(np.asarray(bounds), ords, side="right") - 1
    counts = np.bincount(seg_of, minlength=S)
    first_pos = np.concatenate([[0], np.cumsum(counts)])
    out = {"bounds": bounds, "n_tiles": n_tiles, "launch_end_us": float(us(max(tiles[:, 1].max(), segs[:, :, 1].max())))}
    for s in range(S):
        ts = tiles[first_pos[s] // 64:(first_pos[s + 1] + 63) // 64]
        out[f"tiles_seg{s}"] = {"count": int(len(ts)), "start_us_min": float(us(ts[:, 0].min())),
                                "end_us_median": float(np.median(us(ts[:, 1]))),
                                "end_us_max": float(us(ts[:, 1].max())),
                                "dur_us_median": float(np.median((ts[:, 1] - ts[:, 0]) / 100.0))}
        g = segs[:, s]
        out[f"segment{s}"] = {"start_us_min": float(us(g[:, 0].min())),
                              "start_us_median": float(np.median(us(g[:, 0]))),
                              "start_us_max": float(us(g[:, 0].max())),
                              "end_us_max": float(us(g[:, 1].max())),
                              "dur_us_median": float(np.median((g[:, 1] - g[:, 0]) / 100.0)),
                              "dur_us_p90": float(np.percentile((g[:, 1] - g[:, 0]) / 100.0, 90))}
    # groups whose final segment ends last: what their chain looked like
    last = np.argsort(segs[:, S - 1, 1])[-5:]
    out["latest_groups"] = [{"group": int(gi), "segments_us": [[float(us(segs[gi, s, 0])), float(us(segs[gi, s, 1]))]
                                                             for s in range(S)]} for gi in last]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
