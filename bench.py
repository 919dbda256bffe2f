#!/usr/bin/env python3
"""Benchmark of MirBFT's Actions.Hash hot path on MI355X.

Workload (BASELINE.json configs[1]): synthetic Actions.Hash stream of 2^20
requests x 256 B data (272-byte messages: LE64(client) || LE64(reqNo) || data,
state_machine.go:313-317) plus the dependent BatchSize-20 batch digests
(sequence.go:154-157) computed on device from the device-resident request
digests.  One step = request digests + batch digests for one such stream.
Inputs are generated on device and resident in HBM before the timed region.

Multi-GPU: one process per GPU (torchrun); every rank hashes its own
request range (weak scaling), no collective in the data path; the barrier and
max-over-ranks timing use torch.distributed.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from mirbft_amd import Engine, sharding  # noqa: E402
from mirbft_amd.engine import KERNEL_CHAIN, KERNEL_FUSED, KERNEL_LISTS, KERNEL_MSGS  # noqa: E402

SEED_BASE = 0x6D69726266740000
# Algorithmic work unit: one 64-byte SHA-256 compression = 1384 int32 VALU ops
# (SURVEY.md §8d); gfx950 int32 VALU peak = 256 CU x 4 SIMD x 32 lanes x 2.4 GHz.
OPS_PER_COMPRESSION = 1384
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # 78.64
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    # config id: (data_len, n_requests, batch_size, description)
    2: (256, 1 << 20, 20, "Synthetic Actions.Hash stream: 1M requests x 256 B, BatchSize 20, request + batch digests"),
    3: (4096, 1 << 18, 500, "Large-payload stream: 256K requests x 4 KB, BatchSize 500, VerifyBatch recomputation"),
}


def blocks(L):
    return (np.asarray(L, dtype=np.int64) + 72) >> 6


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=100,
                   help="untimed steps; MI355X needs ~20+ ms of sustained load to reach its working clock")
    p.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    p.add_argument("--variant", type=int, default=0, help="0 = LDS-staged loader, 1 = direct per-lane loads")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU baseline sample (0 disables)")
    p.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive host-API measurement")
    p.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"))
    p.add_argument("--pipeline", default="auto", choices=["auto", "none", "fused", "sequential", "streams"],
                   help="auto: mirsha_pipeline plan, AUTO mode (fused launch for long chains, else request "
                        "kernel then list kernel); none: plain device API (request kernel, then batch kernel); "
                        "fused / sequential / streams: force a plan mode (A/B)")
    p.add_argument("--events-in-timed-loop", type=int, default=1,
                   help="1: per-kernel HIP events inside the timed loop (roofline from the same region); "
                        "0: time the loop bare, then measure kernels in a second identical pass")
    return p.parse_args()


def cpu_baseline(cfg_id, data_len, n_req, bs, seconds):
    """Oracle (C port of processor.go:133-143 with SHA-NI compression, the
    instruction class Go's crypto/sha256 uses on amd64) on the host cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py

    stride = 16 + data_len
    n = min(n_req, 1 << 16)
    n -= n % bs
    arena = oracle_py.gen_requests(SEED_BASE + cfg_id, 0, n, data_len)
    off = np.arange(n, dtype=np.uint64) * stride
    ln = np.full(n, stride, dtype=np.uint32)
    idx, first = sharding.batch_lists(n, bs)
    res = {}
    for threads in (1, min(16, os.cpu_count() or 1)):
        done, t0 = 0, time.perf_counter()
        budget = seconds if threads == 1 else seconds / 3
        while True:
            d = oracle_py.hash_requests(arena, off, ln, threads=threads)
            oracle_py.batch_digests(d, idx, first)
            done += 1
            if time.perf_counter() - t0 >= budget:
                break
        dt = time.perf_counter() - t0
        digests = done * (n + first.size - 1)
        res[threads] = (digests / dt, done, dt)
    v1, done1, dt1 = res[1]
    tp = max(k for k in res)
    return {
        "value": v1,
        "unit": "digests/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{done1} passes x ({n} requests x {stride} B + {first.size - 1} BatchSize-{bs} batch digests), "
                  f"{dt1:.1f} s, oracle C port of processor.go:133-143 (serial Processor), "
                  f"SHA-NI compression (stand-in for Go crypto/sha256 amd64 asm)",
        "pool": {"value": res[tp][0], "threads": tp,
                 "note": "order-preserving ProcessorWorkPool analogue (processor.go:312-361)"},
        "cpu": _cpu_model(),
    }


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    data_len, n, bs, desc = CONFIGS[a.config]
    stride = 16 + data_len
    first_req = rank * n  # weak scaling: each rank its own request range

    eng = Engine(local)
    eng.set_variant(a.variant)
    stream = torch.cuda.current_stream(dev)
    eng.set_stream(stream.cuda_stream)

    d_arena = torch.empty(n * stride, dtype=torch.uint8, device=dev)
    d_off = torch.arange(n, dtype=torch.int64, device=dev) * stride
    d_len = torch.full((n,), stride, dtype=torch.int32, device=dev)
    d_req = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    idx, first = sharding.batch_lists(n, bs)
    nbat = first.size - 1
    d_idx = torch.from_numpy(idx.astype(np.int32)).to(dev)
    d_first = torch.from_numpy(first.astype(np.int32)).to(dev)
    d_bat = torch.empty((nbat, 32), dtype=torch.uint8, device=dev)
    eng.synth_requests_device(SEED_BASE + a.config, first_req, n, data_len, d_arena.data_ptr())
    torch.cuda.synchronize(dev)

    plan = eng.pipeline(n, idx, first, np.full(n, stride), mode=a.pipeline) if a.pipeline != "none" else None

    def step():
        if plan is not None:
            eng.hash_requests_then_batches_device(plan, d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(),
                                                  d_len.data_ptr(), d_req.data_ptr(), d_bat.data_ptr())
            return
        eng.hash_batch_device(d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(), d_len.data_ptr(), None, n,
                              d_req.data_ptr())
        eng.digest_lists_device(d_req.data_ptr(), n, d_idx.data_ptr(), d_first.data_ptr(), nbat, int(first[-1]),
                                d_bat.data_ptr())

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)

    def timed(with_events):
        eng.set_timing(with_events)
        eng.reset_timing()
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        el = time.perf_counter() - t0
        eng.set_timing(False)
        return el

    dt = timed(bool(a.events_in_timed_loop))
    dt_bare = None
    if not a.events_in_timed_loop:
        dt_bare = dt
        timed(True)
    n_msgs, ms_msgs = eng.kernel_time(KERNEL_MSGS)
    n_lists, ms_lists = eng.kernel_time(KERNEL_LISTS)
    n_chain, ms_chain = eng.kernel_time(KERNEL_CHAIN)
    n_fused, ms_fused = eng.kernel_time(KERNEL_FUSED)
    if plan is not None:
        plan.status()  # raises if a fused run's readiness watchdog ever expired

    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # quick self-check of the last step against the CPU oracle on a sample
    check_ok = None
    if rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_py

        k = 256
        arena = oracle_py.gen_requests(SEED_BASE + a.config, first_req, k, data_len)
        want = oracle_py.hash_requests(arena, np.arange(k, dtype=np.uint64) * stride, np.full(k, stride))
        check_ok = bool(np.array_equal(d_req[:k].cpu().numpy(), want))

    # algorithmic totals per step (per rank)
    req_blocks = int(blocks(stride)) * n
    bsz = np.diff(first).astype(np.int64) * 32
    bat_blocks = int(blocks(bsz).sum())
    bytes_hashed = n * stride + int(bsz.sum())
    digests_per_step = n + nbat
    value = digests_per_step * world * a.steps / dt
    gbps = bytes_hashed * world * a.steps / dt / 1e9

    fused = n_fused > 0
    if fused:
        # One persistent launch does the request AND the batch compressions.
        kname, n_k, ms_k, work_blocks = "sha256_fused_paced_kernel", n_fused, ms_fused, req_blocks + bat_blocks
        hbm_bytes = n * stride + n * 32 + int(first[-1]) * 32 + nbat * 32
    else:
        kname, n_k, ms_k, work_blocks = "sha256_msgs_kernel", n_msgs, ms_msgs, req_blocks
        hbm_bytes = n * stride + n * 32
    avg_msgs_ms = ms_k / max(n_k, 1)
    msgs_ms_per_step = ms_k / a.steps  # all launches of the dominant kernel in one step
    avg_lists_ms = (ms_lists + ms_chain) / a.steps  # separate dependent pass device time per step
    achieved_tops = work_blocks * OPS_PER_COMPRESSION / (msgs_ms_per_step * 1e-3) / 1e12
    hbm_gbs = hbm_bytes / (msgs_ms_per_step * 1e-3) / 1e9

    traffic = None
    if os.path.exists(a.traffic_file):
        try:
            tf = json.load(open(a.traffic_file))
            traffic = tf.get(f"config{a.config}", {}).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    pcie = None
    if rank == 0 and world == 1 and not a.no_pcie:
        arena_h = d_arena.cpu().numpy()
        off_h = np.arange(n, dtype=np.uint64) * stride
        len_h = np.full(n, stride, dtype=np.uint32)
        eng.set_stream(None)
        eng.hash_requests_then_batches(arena_h, off_h, len_h, idx, first)  # warm buffers
        reps, t1 = 3, time.perf_counter()
        for _ in range(reps):
            eng.hash_requests_then_batches(arena_h, off_h, len_h, idx, first)
        pdt = (time.perf_counter() - t1) / reps
        pcie = {"digests_per_s": digests_per_step / pdt, "gb_per_s": bytes_hashed / pdt / 1e9,
                "ms_per_call": pdt * 1e3,
                "note": "host API (pageable arena -> HBM -> digests -> host), synchronous"}

    cpu = None
    if rank == 0 and world == 1 and a.cpu_seconds > 0:
        cpu = cpu_baseline(a.config, data_len, n, bs, a.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "SHA-256 digests/s (request + batch digests), Actions.Hash stream",
            "value": value,
            "unit": "digests/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 request stream generated on device, SURVEY.md §8d)",
            "config": {
                "workload": f"config{a.config}: {desc}",
                "requests_per_gpu": n,
                "request_bytes": stride,
                "batch_size": bs,
                "batch_digests_per_gpu": nbat,
                "compressions_per_step_per_gpu": req_blocks + bat_blocks,
                "parallelism": f"request-range shards x{world}, no collective",
                "kernel_variant": ["lds", "direct", "lds_cxx", "direct_cxx"][a.variant],
                "pipeline": a.pipeline if plan is None else f"{a.pipeline} -> {plan.mode_name}",
            },
            "gb_per_s_hashed": gbps,
            "roofline": {
                "bound": "valu",
                "achieved": achieved_tops,
                "peak": VALU_PEAK_TOPS,
                "unit": "TOP/s",
                "frac": achieved_tops / VALU_PEAK_TOPS,
                "traffic": traffic,
                "kernel": kname,
                "avg_launch_ms": avg_msgs_ms,
                "launches_per_step": n_k / a.steps,
                "kernel_ms_per_step": msgs_ms_per_step,
                "work": f"{work_blocks} compressions x {OPS_PER_COMPRESSION} int32 ops per step "
                        f"(over {n_k // a.steps} launch(es))",
                "hbm_algorithmic_gb_per_s": hbm_gbs,
                "hbm_frac": hbm_gbs / HBM_PEAK_GBS,
                "note": "SHA-256 is int32 VALU work (no MFMA shape); hbm/mfma bounds do not apply",
            },
            "batch_kernel_avg_ms": avg_lists_ms,
            "batch_pass": {"none": "sequential batch kernel (plain device API)",
                           "fused": "fused into the request launch (readiness counters, no second kernel)",
                           "sequential": "plan: request kernel then batch kernel",
                           "streams": "chain segments %s on a second stream" % (plan.segments() if plan else None),
                           }[plan.mode_name if plan is not None else "none"],
            "events_in_timed_loop": bool(a.events_in_timed_loop),
            "self_check": check_ok,
            "pcie_inclusive": pcie,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
