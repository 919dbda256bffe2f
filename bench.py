#!/usr/bin/env python3
"""Benchmark of MirBFT's Actions.Hash hot path on MI355X.

Default workload (BASELINE.json configs[1], "config 2"): synthetic Actions.Hash
stream of 2^20 requests x 256 B data (272-byte messages: LE64(client) ||
LE64(reqNo) || data, state_machine.go:313-317) plus the dependent BatchSize-20
batch digests (sequence.go:154-157) computed on device from the
device-resident request digests.  One step = request digests + batch digests
for one such stream (one Ready() cycle's Actions.Hash).

Other configs (--config): 3 = 2^18 x 4 KB requests + BatchSize-500
VerifyBatch digests (batch_tracker.go:147-150); 5 = mixed 64 B - 64 KB
requests (log-uniform octaves), 12.5M per GPU = 10^8 over 8 GPUs.
Inputs are generated on device and resident in HBM before the timed region.
4 = one node's Ready() cycle during a 64-node epoch change: 4096
EpochChangeAck hash requests (64 origins x 64 relaying sources, 61.6 KB
epochChangeHashData payloads of 3847 slices each, stateless.go:311-340) given
as HOST slices, as the Go state machine hands them over; each step is the
host API call (dedup + pack + H2D + kernel + D2H), so this config is
PCIe-inclusive by nature.  A synthetic stand-in: the testengine run that
BASELINE config 4 names needs Go, which this image lacks.

Multi-GPU: one process per GPU; every rank hashes its own request range (weak
scaling), no collective in the data path; the barrier and max-over-ranks
timing use torch.distributed.  `--gpus N` starts the N ranks itself (child
processes, before anything touches a GPU: launch_ranks) unless a launcher
(torchrun) already set WORLD_SIZE, in which case --gpus must equal it.  The
reference scales its hashing with cores the same way, one worker per core
(processor.go:401-408, HashWorkers = runtime.NumCPU()).

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Product imports happen in _import_product(), after the launcher decision:
# the launching parent never loads the engine or touches a device.
torch = None
Engine = MultiEngine = sharding = None
KERNEL_CHAIN = KERNEL_FUSED = KERNEL_LISTS = KERNEL_MSGS = KERNEL_OVERLAP = None


def _import_product():
    global torch, Engine, MultiEngine, sharding
    global KERNEL_CHAIN, KERNEL_FUSED, KERNEL_LISTS, KERNEL_MSGS, KERNEL_OVERLAP
    import torch as _torch

    from mirbft_amd import Engine as _E, MultiEngine as _M, sharding as _s
    from mirbft_amd import engine as _eng

    torch, Engine, MultiEngine, sharding = _torch, _E, _M, _s
    KERNEL_CHAIN, KERNEL_FUSED, KERNEL_LISTS = _eng.KERNEL_CHAIN, _eng.KERNEL_FUSED, _eng.KERNEL_LISTS
    KERNEL_MSGS, KERNEL_OVERLAP = _eng.KERNEL_MSGS, _eng.KERNEL_OVERLAP

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
    5: (None, 12_500_000, 0, "Mixed-size stream: 64 B - 64 KB requests (log-uniform octaves), "
                             "12.5M per GPU (10^8 over 8 GPUs), request-range sharded"),
    4: (None, 4096, 0, "Epoch-change cycle of a 64-node network: 64 origins x 64 relaying sources "
                       "EpochChangeAck digests (61.6 KB payloads, host slices), content-addressed dedup"),
}


def blocks(L):
    return (np.asarray(L, dtype=np.int64) + 72) >> 6


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="ranks (one process per GPU); without a launcher's WORLD_SIZE, bench.py starts them itself")
    p.add_argument("--launch-check", action="store_true",
                   help="launcher plumbing only (CPU tests): ranks rendezvous over gloo, barrier, gather their "
                        "request ranges, rank 0 prints the line with value null; no device, no hashing")
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=100,
                   help="untimed steps; MI355X needs ~20+ ms of sustained load to reach its working clock")
    p.add_argument("--config", type=int, default=2, choices=[1] + sorted(CONFIGS),
                   help="BASELINE config (1 = small-cycle latency of the host API)")
    p.add_argument("--requests", type=int, default=0, help="requests per GPU (0 = the config's)")
    p.add_argument("--variant", type=int, default=0, choices=[0, 1, 4, 5, 6, 10],
                   help="0 = LDS-staged loader (latency forms for small launches), 1 = direct per-lane loads, "
                        "4 = low-occupancy kernel, 5 = LDS kernel only, 6 = pair kernel")
    p.add_argument("--windows", action="store_true",
                   help="config 5: hash in <= 4 GiB windows (one launch each) instead of one 64-bit-addressed launch")
    p.add_argument("--prewarm-ms", type=float, default=400.0,
                   help="after the warm-up steps, keep running untimed steps until this much wall time has passed: "
                        "the clock needs tens of ms of sustained load to settle, and the driver's --warmup 5 is "
                        "~1.5 ms (reported as prewarm_ms / prewarm_steps)")
    p.add_argument("--probe-iters", type=int, default=128,
                   help="clock probe after the timed region (compressions per wave; 0 disables)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU baseline sample (0 disables)")
    p.add_argument("--dedup", type=int, default=1, help="config 4: 1 = mirsha_hash_slices_dedup, 0 = plain")
    p.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive host-API measurement")
    p.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="PMC traffic per launch, keyed by kernel_source_key(); written by profiles/profile.sh")
    p.add_argument("--no-overlap-extra", dest="overlap_extra", action="store_false",
                   help="skip the overlapped-cycles figure (configs 2/3 with a sequential plan)")
    p.add_argument("--no-config3-leg", dest="config3_leg", action="store_false",
                   help="config 2 runs: skip the config-3 leg (fused step, overlapped cycles, sequential request "
                        "kernel) measured after the headline")
    p.add_argument("--pipeline", default="auto", choices=["auto", "none", "fused", "sequential", "overlap"],
                   help="auto: mirsha_pipeline plan, AUTO mode (fused launch for long chains, else request "
                        "kernel then list kernel); none: plain device API (request kernel, then batch kernel); "
                        "fused / sequential: force a plan mode (A/B)")
    p.add_argument("--timed-kernels", default="dominant", choices=["dominant", "all"],
                   help="kernels with HIP events inside the timed loop: the dominant (roofline) kernel only, "
                        "or every kernel (each timed launch adds two event records to the stream); with "
                        "'dominant' the other kernels are timed in a second, unreported-as-value pass")
    p.add_argument("--events-in-timed-loop", type=int, default=1,
                   help="1: per-kernel HIP events inside the timed loop (roofline from the same region); "
                        "0: time the loop bare, then measure kernels in a second identical pass")
    p.add_argument("--repeat-regions", type=int, default=5,
                   help="after the headline, time the same --steps region this many more times (bare) and report "
                        "their per-step median beside the value (SURVEY.md §8d: median over repeats)")
    p.add_argument("--event-every", type=int, default=4,
                   help="inside the timed loop the dominant kernel's HIP events ride on every k-th step's launch "
                        "(bound to its dispatch, hipExtLaunchKernel): an event-bound launch adds ~5 us of stream "
                        "time on gfx950 (profiles/r06h), so the wall time carries 1/k of it; the kernel average "
                        "is over the sampled launches of the same timed region")
    return p.parse_args()


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py  # test infrastructure: CPU baseline and self-check only

    return oracle_py


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_facts():
    """What the CPU baseline ran on: the reference's ProcessorWorkPool default is
    HashWorkers = runtime.NumCPU() (processor.go:406-408), and Go's NumCPU is the
    size of the process's CPU affinity mask."""
    facts = {"os_cpu_count": os.cpu_count()}
    try:
        facts["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        facts["affinity_cpus"] = os.cpu_count()
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        facts["cgroup_cpu_quota"] = None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        facts["cgroup_cpu_quota"] = None
    try:
        facts["sha_ni"] = bool(_oracle().has_shani())
    except Exception:  # noqa: BLE001 - informational only
        facts["sha_ni"] = None
    return facts


def pool_threads():
    """HashWorkers = runtime.NumCPU() (processor.go:406-408): the affinity mask."""
    return _cpu_facts()["affinity_cpus"] or 1


def kernel_source_key(variant):
    """Identity of the kernel build whose PMC traffic a profile recorded: the
    sha256 of the device sources plus the variant (the .so is not in git, the
    sources are)."""
    import hashlib

    h = hashlib.sha256()
    for f in ("mirsha_kernels.hip", "mirsha_kernels.h", "sha256_device.h", "sha256_rounds_asm.h"):
        with open(os.path.join(ROOT, "mirbft_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    h.update(str(int(variant)).encode())
    return h.hexdigest()[:16]


def lookup_traffic(path, key, config, kernel):
    """hbm_bytes_per_launch of the dominant kernel for this build, or None."""
    try:
        tf = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    for e in tf.get("entries", []):
        if (e.get("key") == key and int(e.get("config", -1)) == int(config)
                and e.get("kernel", "sha256_msgs_kernel") == kernel):
            return e.get("hbm_bytes_per_launch"), e
    return None, None


def _time_cpu(fn, seconds, threads_list):
    res = {}
    for threads in threads_list:
        done, t0 = 0, time.perf_counter()
        budget = seconds if threads == 1 else seconds / 3
        while True:
            fn(threads)
            done += 1
            if time.perf_counter() - t0 >= budget:
                break
        res[threads] = (done, time.perf_counter() - t0)
    return res


def event_steps(steps, every):
    """Steps of a timed region whose dominant launch carries HIP events:
    every `every`-th from the `every`-th on (never step 0, the first launch
    after the idle sync, whose dispatch starts late: profiles/r06k); `every`
    is clamped to the region so at least one step is sampled."""
    every = max(1, min(int(every), int(steps)))
    return [i for i in range(steps) if i % every == every - 1]


def check_windows(n_batches, batch_size, seed, per_window=256):
    """Batch ranges [b0, b1) the self-check samples: the first window, the
    last (it ends with the final batch, which is short when BatchSize does not
    divide the request count) and 4 random ones, each ~per_window requests."""
    k = max(1, per_window // max(batch_size, 1))
    if n_batches <= 0:
        return []
    rng = np.random.default_rng(seed)
    hi = max(n_batches - k, 0)
    starts = {0, hi} | {int(x) for x in rng.integers(0, hi + 1, size=4)}
    return [(b0, min(b0 + k, n_batches)) for b0 in sorted(starts)]


def check_batch_windows(seed, first_req, data_len, idx, first, req_digests, bat_digests):
    """Compare request digests [first[b0], first[b1]) and batch digests
    [b0, b1) of every check_windows window with the oracle (generator ->
    oracle_hash_requests -> oracle_batch_digests).  req_digests / bat_digests:
    (n, 32) / (n_batches, 32) host arrays of the rank's own range."""
    o = _oracle()
    stride = 16 + data_len
    ok = True
    for b0, b1 in check_windows(first.size - 1, int(first[1] - first[0]) if first.size > 1 else 1, first_req + 17):
        i0, i1 = int(first[b0]), int(first[b1])
        arena = o.gen_requests(seed, first_req + i0, i1 - i0, data_len)
        want = o.hash_requests(arena, np.arange(i1 - i0, dtype=np.uint64) * stride, np.full(i1 - i0, stride))
        ok = ok and bool(np.array_equal(req_digests[i0:i1], want))
        wb = o.batch_digests(want, idx[i0:i1].astype(np.int64) - i0, first[b0:b1 + 1].astype(np.int64) - i0)
        ok = ok and bool(np.array_equal(bat_digests[b0:b1], wb))
    return ok


class BatchWorkload:
    """Configs 2 and 3: a dense stream of equal-size requests + batch lists."""

    def __init__(self, a, eng, dev, rank):
        self.a, self.eng = a, eng
        self.data_len, n0, self.bs, self.desc = CONFIGS[a.config]
        self.n = n = a.requests or n0
        self.stride = stride = 16 + self.data_len
        self.seed = SEED_BASE + a.config
        self.first_req = rank * n  # weak scaling: each rank its own request range
        self.d_arena = torch.empty(n * stride, dtype=torch.uint8, device=dev)
        self.d_off = torch.arange(n, dtype=torch.int64, device=dev) * stride
        self.d_len = torch.full((n,), stride, dtype=torch.int32, device=dev)
        self.d_req = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        self.idx, self.first = sharding.batch_lists(n, self.bs)
        self.nbat = self.first.size - 1
        self.d_idx = torch.from_numpy(self.idx.astype(np.int32)).to(dev)
        self.d_first = torch.from_numpy(self.first.astype(np.int32)).to(dev)
        self.d_bat = torch.empty((self.nbat, 32), dtype=torch.uint8, device=dev)
        eng.synth_requests_device(self.seed, self.first_req, n, self.data_len, self.d_arena.data_ptr())
        # overlap: each step is ONE launch hashing this cycle's requests and the
        # previous cycle's batches (mirsha_pipeline_overlap_device) on a
        # sequential plan; request digests alternate between two buffers.
        self.overlap = a.pipeline == "overlap"
        pmode = "auto" if self.overlap else a.pipeline
        self.plan = (eng.pipeline(n, self.idx, self.first, np.full(n, stride), mode=pmode)
                     if a.pipeline != "none" else None)
        self.d_reqs = [self.d_req, torch.empty_like(self.d_req)] if self.overlap else None
        self.cycle = 0
        self.req_blocks = int(blocks(stride)) * n
        bsz = np.diff(self.first).astype(np.int64) * 32
        self.bat_blocks = int(blocks(bsz).sum())
        self.bytes_hashed = n * stride + int(bsz.sum())
        self.digests = n + self.nbat

    def step(self):
        e = self.eng
        if self.overlap:
            cur, prev = self.d_reqs[self.cycle % 2], self.d_reqs[(self.cycle + 1) % 2]
            e.pipeline_overlap_device(self.plan, self.d_arena.data_ptr(), self.d_arena.numel(), self.d_off.data_ptr(),
                                      self.d_len.data_ptr(), cur.data_ptr(),
                                      prev.data_ptr() if self.cycle else 0, self.d_bat.data_ptr())
            self.d_req = cur  # the last cycle's request digests (self_check)
            self.cycle += 1
            return
        if self.plan is not None:
            e.hash_requests_then_batches_device(self.plan, self.d_arena.data_ptr(), self.d_arena.numel(),
                                                self.d_off.data_ptr(), self.d_len.data_ptr(), self.d_req.data_ptr(),
                                                self.d_bat.data_ptr())
            return
        e.hash_batch_device(self.d_arena.data_ptr(), self.d_arena.numel(), self.d_off.data_ptr(),
                            self.d_len.data_ptr(), None, self.n, self.d_req.data_ptr())
        e.digest_lists_device(self.d_req.data_ptr(), self.n, self.d_idx.data_ptr(), self.d_first.data_ptr(),
                              self.nbat, int(self.first[-1]), self.d_bat.data_ptr())

    def after(self):
        if self.plan is not None:
            self.plan.status()  # raises if a fused run's readiness watchdog ever expired

    def dominant(self):
        """(kernel name, launches, ms, compressions, algorithmic HBM bytes) of the dominant kernel."""
        n_o, ms_o = self.eng.kernel_time(KERNEL_OVERLAP)
        if n_o:
            # One launch: this cycle's request compressions + the previous cycle's batch chains.
            hbm = self.n * (self.stride + 32 + 12) + int(self.first[-1]) * 32 + self.nbat * 32
            return "sha256_msgs_overlap_kernel", n_o, ms_o, self.req_blocks + self.bat_blocks, hbm
        n_f, ms_f = self.eng.kernel_time(KERNEL_FUSED)
        if n_f:
            # One launch does the request AND the batch compressions.
            hbm = self.n * (self.stride + 32 + 12) + int(self.first[-1]) * 32 + self.nbat * 32
            return "sha256_fused_paced_kernel", n_f, ms_f, self.req_blocks + self.bat_blocks, hbm
        n_m, ms_m = self.eng.kernel_time(KERNEL_MSGS)
        # message bytes + digest + its off (u64) and len (u32) entries
        return "sha256_msgs_kernel", n_m, ms_m, self.req_blocks, self.n * (self.stride + 32 + 12)

    def batch_ms(self):
        return self.eng.kernel_time(KERNEL_LISTS)[1] + self.eng.kernel_time(KERNEL_CHAIN)[1]

    def self_check(self):
        """This rank's last step against the oracle: request and batch digests
        of batch-aligned windows (check_windows: the first, the last -- which
        holds the final, possibly partial batch -- and 4 random ones)."""
        torch.cuda.synchronize(self.d_req.device)
        return check_batch_windows(self.seed, self.first_req, self.data_len, self.idx, self.first,
                                   self.d_req.cpu().numpy(), self.d_bat.cpu().numpy())

    def pcie(self):
        n, stride = self.n, self.stride
        arena_h = self.d_arena.cpu().numpy()
        off_h = np.arange(n, dtype=np.uint64) * stride
        len_h = np.full(n, stride, dtype=np.uint32)
        self.eng.set_stream(None)

        # Result buffers reused across calls, as the cgo binding reuses its
        # digest buffer: a fresh 32 MiB array per call adds
        # ~30 ms of first-touch page faults.
        req_h = np.empty((n, 32), dtype=np.uint8)
        bat_h = np.empty((self.nbat, 32), dtype=np.uint8)

        def rate(arena):
            def call():
                self.eng.hash_requests_then_batches(arena, off_h, len_h, self.idx, self.first, out=req_h,
                                                    batch_out=bat_h)

            call()  # warm device buffers
            t = []
            for _ in range(10):
                t1 = time.perf_counter()
                call()
                t.append(time.perf_counter() - t1)
            return float(np.median(t)), [round(x * 1e3, 3) for x in t]

        pdt, pcalls = rate(arena_h)
        pprof = self.eng.host_profile()
        pinned = self.eng.host_empty(arena_h.size)
        pinned[:] = arena_h
        qdt, qcalls = rate(pinned)
        qprof = self.eng.host_profile()
        self.eng.set_stream(torch.cuda.current_stream(self.d_arena.device).cuda_stream)  # back to the steps' stream
        return {"digests_per_s": self.digests / pdt, "gb_per_s": self.bytes_hashed / pdt / 1e9,
                "ms_per_call": pdt * 1e3, "calls_ms": pcalls, "host_phases_ms": pprof,
                "note": "host API (pageable arena -> HBM -> digests -> reused host buffers), synchronous; "
                        "median of 10 calls after one warm-up call; host_phases_ms = the last call's phases",
                "pinned_arena": {"digests_per_s": self.digests / qdt, "gb_per_s": self.bytes_hashed / qdt / 1e9,
                                 "ms_per_call": qdt * 1e3, "calls_ms": qcalls, "host_phases_ms": qprof,
                                 "note": "the same call on an arena from mirsha_host_alloc (page-locked)"}}

    def multi_device(self):
        """The multi-GPU drop-in (mirsha_hash_arena_multi, INTEGRATION.md's
        GPUHasherMulti): the config's requests from host memory, cut into
        contiguous ranges of equal bytes, one per listed device, each over its
        own PCIe link and stream.  Devices: every visible GPU when there are
        several, else two contexts on GPU 0 (one link: the mechanics and the
        per-device phases, not a speed-up).  Digests checked against the
        oracle on samples at both ends and on both sides of every cut."""
        ndev = torch.cuda.device_count()
        devices = list(range(ndev)) if ndev > 1 else [0, 0]
        n, stride = self.n, self.stride
        arena_h = self.d_arena.cpu().numpy()
        off_h = np.arange(n, dtype=np.uint64) * stride
        len_h = np.full(n, stride, dtype=np.uint32)
        out = np.empty((n, 32), dtype=np.uint8)
        m = MultiEngine(devices)
        try:
            m.set_variant(self.a.variant)

            def rate(arena):
                m.hash_arena(arena, off_h, len_h, out=out)  # warm device buffers
                t = []
                for _ in range(5):
                    t1 = time.perf_counter()
                    m.hash_arena(arena, off_h, len_h, out=out)
                    t.append(time.perf_counter() - t1)
                return float(np.median(t)), [round(x * 1e3, 3) for x in t]

            pdt, pcalls = rate(arena_h)
            pinned = m.host_empty(arena_h.size)
            pinned[:] = arena_h
            qdt, qcalls = rate(pinned)
            cut = m.last_cut()
            # oracle samples: the first and last requests and both sides of every cut
            o, k = _oracle(), 128
            starts = sorted({0, max(n - k, 0)} | {min(max(c - k // 2, 0), max(n - k, 0)) for c in cut[1:-1]})
            ok = True
            for i0 in starts:
                cnt = min(k, n - i0)
                sample = o.gen_requests(self.seed, self.first_req + i0, cnt, self.data_len)
                want = o.hash_requests(sample, np.arange(cnt, dtype=np.uint64) * stride, np.full(cnt, stride))
                ok = ok and bool(np.array_equal(out[i0:i0 + cnt], want))
            phases = [{"device": d, "requests": cut[k + 1] - cut[k], "host_phases_ms": m.host_profile(k)}
                      for k, d in enumerate(devices)]
        finally:
            m.close()
        req_bytes = n * stride
        return {"devices": devices, "digests_per_s": n / qdt, "gb_per_s": req_bytes / qdt / 1e9,
                "ms_per_call": qdt * 1e3, "calls_ms": qcalls, "per_device": phases,
                "pageable": {"digests_per_s": n / pdt, "gb_per_s": req_bytes / pdt / 1e9, "ms_per_call": pdt * 1e3,
                             "calls_ms": pcalls},
                "self_check": ok,
                "note": "mirsha_hash_arena_multi, request digests only (no lists), page-locked arena from "
                        "mirsha_multi_host_alloc (headline) and pageable; median of 5 calls after a warm-up; "
                        "per_device = the last pinned call's range and phases per device context"
                        + ("" if ndev > 1 else "; one GPU visible: two contexts share its link")}

    def cgo_path(self):
        """The Go binding's HashBatch end to end, slices -> digests
        (tests/c/cgo_path.c, a separate process with no Python: request
        Data as 3 heap slices each; a persistent 15-worker pool stands in for
        the goroutines).  Config 2 at full size.  Legs: 'parallel' =
        INTEGRATION.md's HashBatch (32 MiB chunks packed into the pinned arena
        while the calling thread submits the previous one, mirsha_submit_batch), 'onecall' =
        round 4's (pack all, then one mirsha_hash_batch), 'serial' = one
        goroutine packs, 'lib' = mirsha_hash_slices, 'multi' = the chunked
        form over every device (mirsha_submit_arena_multi)."""
        exe = os.path.join(ROOT, "tests", "c", "build", "cgo_path")
        if not os.path.exists(exe):
            return {"note": f"{exe} not built (__graft_entry__.build())"}
        # 15 packing workers + the submitting thread = the GPU box's 16-CPU share
        # "nt": the workers stream the arena with non-temporal stores (INTEGRATION.md streamPack)
        r = subprocess.run([exe, str(self.n), str(self.data_len), "15", "7", "32", "nt"], capture_output=True,
                           text=True, timeout=300)
        if r.returncode != 0:
            return {"error": r.stderr[-500:]}
        out = json.loads(r.stdout.splitlines()[-1])
        out.pop("sample", None)
        out["note"] = ("INTEGRATION.md GPUHasher.HashBatch made from C: 'parallel' = the chunked form (15 workers "
                       "pack chunk k+1 with non-temporal stores while the caller submits chunk k, "
                       "mirsha_submit_batch: DMA / kernel / D2H on "
                       "three streams; digests DMA'd into a pinned buffer, copied to the Go-owned result by the "
                       "workers), 'onecall' = pack "
                       "everything then one mirsha_hash_batch, 'serial' = one goroutine packs, 'lib' = "
                       "mirsha_hash_slices on C slice arrays, 'multi' = the chunked form over every visible device "
                       "(device 0 twice on one GPU); median of 7 calls, PCIe included, every leg's digests equal")
        return out

    def cpu_baseline(self, seconds):
        """Oracle (C port of processor.go:133-143) on the host cores: the
        serial Processor on one core with SHA-NI compression (the headline), the
        same with the portable scalar FIPS 180-4 compression (`go114_class`:
        the reference pins Go 1.13/1.14, .travis.yml:5-6 and go.mod:3, whose
        amd64 crypto/sha256 has no SHA-NI path -- Go added one in 1.21 -- but
        an AVX2/BMI2 block function), and the order-preserving
        ProcessorWorkPool analogue with HashWorkers = NumCPU() (the reference
        default, processor.go:406-408) and with the cgroup quota.  SHA-NI is
        the headline because it is the FASTER CPU figure: the conservative
        baseline for the GPU."""
        o = _oracle()
        stride, bs = self.stride, self.bs
        n = min(self.n, 1 << 16)
        n -= n % bs
        arena = o.gen_requests(self.seed, 0, n, self.data_len)
        off = np.arange(n, dtype=np.uint64) * stride
        ln = np.full(n, stride, dtype=np.uint32)
        idx, first = sharding.batch_lists(n, bs)

        def one(threads):
            d = o.hash_requests(arena, off, ln, threads=threads)
            o.batch_digests(d, idx, first)

        res = _time_cpu(one, seconds, (1,))
        per = n + first.size - 1
        done1, dt1 = res[1]
        facts = _cpu_facts()
        # Scalar FIPS compression on the same sample, one core (Go 1.14 class).
        o.force_impl(0)
        try:
            ds, dts = _time_cpu(one, seconds / 4, (1,))[1]
        finally:
            o.force_impl(-1)
        go114 = {"value": ds * per / dts, "unit": "digests/s", "cores": 1,
                 "sample": f"{ds} passes of the headline sample, {dts:.1f} s",
                 "note": "portable scalar FIPS 180-4 compression (gcc -O2), no SHA-NI: the instruction class of "
                         "the reference's Go 1.13/1.14 crypto/sha256 on amd64 (.travis.yml:5-6, go.mod:3), whose "
                         "AVX2/BMI2 block function vectorises the message schedule and has no SHA-NI path "
                         "(Go added SHA-NI in 1.21)"}
        # BASELINE.md's labelled stand-in: the same loop through OpenSSL EVP
        # (oracle/evp_loop.c: three Writes per request, one per RequestAck
        # digest), on the same sample, 1 core; then the pool legs below.
        def evp(threads, arena=arena, off=off, ln=ln, idx=idx, first=first):
            d = o.evp_hash_requests(arena, off, ln, threads=threads)
            o.evp_batch_digests(d, idx, first)

        try:  # an extra leg: a missing libcrypto is reported in the line, not fatal to it
            evp_ok = bool(np.array_equal(o.evp_hash_requests(arena[: 64 * stride], off[:64], ln[:64]),
                                         o.hash_requests(arena[: 64 * stride], off[:64], ln[:64])))
            de, dte = _time_cpu(evp, seconds / 4, (1,))[1]
            openssl = {"value": de * per / dte, "unit": "digests/s", "cores": 1,
                       "label": "OpenSSL stand-in for Go crypto/sha256",
                       "openssl": o.evp_version(), "matches_oracle": evp_ok,
                       "sample": f"{de} passes of the headline sample, {dte:.1f} s",
                       "note": "BASELINE.md CPU-baseline plan: processor.go:133-143 with EVP_DigestInit_ex2 / "
                               "EVP_DigestUpdate per HashRequest.Data slice (3 per request, "
                               "state_machine.go:313-317) / EVP_DigestFinal_ex; batch digests one Update per "
                               "RequestAck digest (oracle/evp_loop.c)"}
        except Exception as e:  # noqa: BLE001
            openssl = {"error": f"{type(e).__name__}: {e}"}
        # Pool legs on a larger sample (whole config up to 2^20 requests), so
        # per-pass thread start-up is noise; batch digests single-threaded, as
        # the state machine consumes them (processResults, state_machine.go:377-433).
        npool = min(self.n, 1 << 20)
        npool -= npool % bs
        parena = o.gen_requests(self.seed, 0, npool, self.data_len)
        poff = np.arange(npool, dtype=np.uint64) * stride
        pln = np.full(npool, stride, dtype=np.uint32)
        pidx, pfirst = sharding.batch_lists(npool, bs)
        pper = npool + pfirst.size - 1
        legs = {}
        for name, t in (("numcpu", facts["affinity_cpus"] or 1),
                        ("quota", int(facts["cgroup_cpu_quota"] or 0))):
            if t < 2 or t in [v["threads"] for v in legs.values()]:
                continue

            def pool(threads):
                d = o.hash_requests(parena, poff, pln, threads=threads)
                o.batch_digests(d, pidx, pfirst)

            r = _time_cpu(pool, seconds / 3, (t,))[t]
            legs[name] = {"value": r[0] * pper / r[1], "threads": t,
                          "sample": f"{r[0]} passes x {npool} requests + {pfirst.size - 1} batch digests, {r[1]:.1f} s"}
            if "error" not in openssl:
                re = _time_cpu(lambda th: evp(th, parena, poff, pln, pidx, pfirst), seconds / 6, (t,))[t]
                openssl.setdefault("pool", {})[name] = {"value": re[0] * pper / re[1], "threads": t,
                                                        "sample": f"{re[0]} passes of the pool sample, "
                                                                  f"{re[1]:.1f} s"}
        return {
            "value": done1 * per / dt1, "unit": "digests/s", "cores": 1, "kind": "port",
            "sample": f"{done1} passes x ({n} requests x {stride} B + {first.size - 1} BatchSize-{bs} batch "
                      f"digests), {dt1:.1f} s, oracle C port of processor.go:133-143 (serial Processor), "
                      f"SHA-NI compression (faster than the reference's Go 1.14 crypto/sha256, which has no "
                      f"SHA-NI path: a conservative baseline; the Go 1.14-class figure is go114_class)",
            "go114_class": go114,
            "openssl_evp": openssl,
            "pool": {**legs,
                     "note": "order-preserving ProcessorWorkPool analogue (processor.go:312-361): workers pull "
                             "requests from a shared counter; numcpu = HashWorkers = runtime.NumCPU() = the affinity "
                             "mask (processor.go:406-408), quota = the container's CPU quota"},
            "cpu": _cpu_model(),
            **facts,
        }

    def config_fields(self):
        return {"requests_per_gpu": self.n, "request_bytes": self.stride, "batch_size": self.bs,
                "batch_digests_per_gpu": self.nbat,
                "compressions_per_step_per_gpu": self.req_blocks + self.bat_blocks,
                "pipeline": self.a.pipeline if self.plan is None else f"{self.a.pipeline} -> {self.plan.mode_name}",
                }

    def overlap_cycles(self):
        """The same plan as overlapped cycles (mirsha_pipeline_overlap_device):
        ONE launch per cycle hashes the cycle's requests and the previous
        cycle's batches, as a stream of Ready() cycles pipelines (the state
        machine batches digests of earlier cycles).  Measured after the
        headline steps on rank 0: --steps launches with the kernel's HIP
        events on (bound to each dispatch), wall time and kernel time from that
        ONE pass (kernel <= wall holds by construction)."""
        if self.plan is None or self.overlap:
            return None
        timer = KERNEL_FUSED if self.plan.mode_name == "fused" else KERNEL_OVERLAP
        e, steps = self.eng, self.a.steps
        d_reqs = [self.d_req, torch.empty_like(self.d_req)]
        state = {"i": 0}

        def launch():
            i = state["i"]
            e.pipeline_overlap_device(self.plan, self.d_arena.data_ptr(), self.d_arena.numel(), self.d_off.data_ptr(),
                                      self.d_len.data_ptr(), d_reqs[i % 2].data_ptr(),
                                      d_reqs[(i + 1) % 2].data_ptr() if i else 0, self.d_bat.data_ptr())
            state["i"] = i + 1

        dev = self.d_req.device
        for _ in range(max(self.a.warmup, 2)):
            launch()
        torch.cuda.synchronize(dev)
        e.set_timing_mask([timer])
        e.set_timing(True)
        e.reset_timing()
        # Events on EVERY launch here (bound to the dispatches): the kernel
        # average is then over the same launches as the wall time, so kernel
        # <= wall holds (a sampled average need not, profiles/r06l); the
        # events' dispatch cost (~5 us per launch, profiles/r06h) stays in this
        # leg's wall time.
        t0 = time.perf_counter()
        for _ in range(steps):
            launch()
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        e.set_timing(False)
        n_o, ms_o = e.kernel_time(timer)
        e.set_timing_mask(range(32))
        kms = ms_o / max(n_o, 1)
        work = (self.req_blocks + self.bat_blocks) * OPS_PER_COMPRESSION
        tops = work / (kms * 1e-3) / 1e12
        step_tops = work / (dt / steps) / 1e12
        return {"digests_per_s": self.digests * steps / dt, "ms_per_step": dt / steps * 1e3,
                "kernel": {KERNEL_FUSED: "sha256_fused_paced_kernel"}.get(timer, "sha256_msgs_overlap_kernel"),
                "avg_launch_ms": kms, "frac": tops / VALU_PEAK_TOPS, "step_frac": step_tops / VALU_PEAK_TOPS,
                "note": "one launch per cycle: this cycle's requests + the previous cycle's batch chains "
                        "(mirsha_pipeline_overlap_device, on this plan), steady state of a cycle stream; "
                        "frac = both over the kernel's event time, step_frac = both over ms_per_step; "
                        "one pass: wall time and the events of every launch (dispatch-bound)"}

    def extra(self):
        mode = self.plan.mode_name if self.plan is not None else "none"
        if self.overlap:
            return {"batch_pass": "overlapped: the previous cycle's batch chains in each cycle's request launch"}
        return {"batch_kernel_avg_ms": getattr(self, "batch_ms_timed", 0.0) / self.a.steps,
                "batch_pass": {"none": "sequential batch kernel (plain device API)",
                               "fused": "fused into the request launch (readiness counters, no second kernel)",
                               "sequential": "plan: request kernel then batch kernel"}[mode],
                "overlap_cycles": getattr(self, "ovl", None)}


class MixedWorkload:
    """Config 5: 64 B - 64 KB requests packed densely in HBM (~123 GB per GPU at
    12.5M requests), hashed in ONE launch (64-bit per-lane addressing) in a
    global longest-first length-bucketed order, so the long chains start first
    and the launch's tail is short messages; --windows: <= 4 GiB origin-order
    windows, one launch each (A/B)."""

    def __init__(self, a, eng, dev, rank, world=1):
        self.a, self.eng = a, eng
        _, n0, _, self.desc = CONFIGS[5]
        per_rank = a.requests or n0
        self.seed = SEED_BASE + 5
        # One global stream of world x per_rank requests, cut into `world`
        # contiguous request ranges of equal compression count by the
        # block-balanced sharder (sharding.shard_ranges with lengths): at
        # N = 8 that is BASELINE config 5's 10^8-request stream.
        g = world * per_rank
        d_all = torch.empty(g, dtype=torch.int32, device=dev)
        eng.synth_mixed_lengths_device(self.seed, 0, g, d_all.data_ptr())
        eng.sync()
        lo, hi = sharding.shard_ranges(g, world, 1, d_all.cpu().numpy().view(np.uint32))[rank]
        n = hi - lo
        self.first_req, self.n = lo, n
        self.global_requests = g
        d_len = d_all[lo:hi].clone()
        del d_all
        self.ln = d_len.cpu().numpy().view(np.uint32)
        self.off = np.zeros(n, dtype=np.uint64)
        np.cumsum(self.ln[:-1], out=self.off[1:])
        self.total = int(self.off[-1]) + int(self.ln[-1])
        if a.windows:
            self.wins = sharding.arena_windows(self.off, self.ln)
        else:
            self.wins = [(0, n, 0)]
        offrel = self.off.copy()
        for i0, i1, base in self.wins:
            offrel[i0:i1] -= np.uint64(base)
        order = sharding.window_orders(self.ln, self.wins)
        self.d_len = d_len
        self.d_off = torch.from_numpy(self.off.view(np.int64)).to(dev)
        self.d_offrel = torch.from_numpy(offrel.view(np.int64)).to(dev) if a.windows else self.d_off
        self.d_order = torch.from_numpy(order.view(np.int32)).to(dev)
        self.d_arena = torch.empty(self.total + 256, dtype=torch.uint8, device=dev)
        self.d_req = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        eng.synth_mixed_device(self.seed, self.first_req, n, self.d_off.data_ptr(), self.d_arena.data_ptr())
        eng.sync()
        self.req_blocks = int(blocks(self.ln).sum())
        self.bytes_hashed = self.total
        self.digests = n
        self.plan = None

    def step(self):
        e = self.eng
        ap, op, lp = self.d_arena.data_ptr(), self.d_offrel.data_ptr(), self.d_len.data_ptr()
        rp, qp = self.d_order.data_ptr(), self.d_req.data_ptr()
        for i0, i1, base in self.wins:
            span = int(self.off[i1 - 1]) + int(self.ln[i1 - 1]) - base
            e.hash_batch_device(ap + base, span, op + 8 * i0, lp + 4 * i0, rp + 4 * i0, i1 - i0, qp + 32 * i0)

    def after(self):
        pass

    def dominant(self):
        n_m, ms_m = self.eng.kernel_time(KERNEL_MSGS)
        return "sha256_msgs_kernel", n_m, ms_m, self.req_blocks, self.total + 32 * self.n

    def self_check(self):
        o = _oracle()
        rng = np.random.default_rng(5 + self.first_req)
        ends = np.r_[np.arange(min(8, self.n)), np.arange(max(self.n - 8, 0), self.n)]  # the range's first / last
        ids = np.unique(np.r_[ends, rng.choice(self.n, size=min(256, self.n), replace=False)])
        arena, off, ln = o.gen_mixed(self.seed, ids + self.first_req)
        if not np.array_equal(ln, self.ln[ids]):
            return False
        want = o.hash_requests(arena, off, ln)
        got = self.d_req[torch.from_numpy(ids.astype(np.int64)).to(self.d_req.device)].cpu().numpy()
        return bool(np.array_equal(got, want))

    def pcie(self):
        return None  # ~123 GB per GPU: the host API path is not measured for this config

    def cpu_baseline(self, seconds):
        o = _oracle()
        # a fixed 10^6-request prefix of the same stream,
        # generated into host RAM first (~9.4 GB), its rate reported (never
        # extrapolated to the 10^8 total)
        k = min(self.n, 1_000_000)
        arena, off, ln = o.gen_mixed(self.seed, np.arange(k, dtype=np.uint64))
        res = _time_cpu(lambda t: o.hash_requests(arena, off, ln, threads=t), seconds, (1, pool_threads()))
        done1, dt1 = res[1]
        tp = max(res)
        return {
            "value": done1 * k / dt1, "unit": "digests/s", "cores": 1, "kind": "port",
            "gb_per_s": done1 * int(ln.sum()) / dt1 / 1e9,
            "sample": f"{done1} passes x {k} mixed requests ({int(ln.sum()) / 1e6:.0f} MB), {dt1:.1f} s, oracle C "
                      f"port of processor.go:133-143, SHA-NI compression",
            "pool": {"value": res[tp][0] * k / res[tp][1], "threads": tp},
            "cpu": _cpu_model(),
            **_cpu_facts(),
        }

    def config_fields(self):
        return {"requests_per_gpu": self.n, "global_requests": self.global_requests,
                "sharding": "sharding.shard_ranges(global stream, world, lengths): contiguous request ranges "
                            "of equal compression count, no collective",
                "first_request_of_rank": self.first_req, "arena_gb_per_gpu": self.total / 1e9,
                "mean_request_bytes": self.total / self.n, "launches_per_step": len(self.wins),
                "addressing": "4 GiB windows" if self.a.windows else "one launch, 64-bit per-lane addresses",
                "compressions_per_step_per_gpu": self.req_blocks}

    def extra(self):
        return {}


class EpochChangeWorkload:
    """Config 4 (see the module docstring): host-slice requests through the
    host API, with content-addressed dedup (mirsha_hash_slices_dedup)."""

    N_NODES, N_CP, N_P, N_Q = 64, 3, 640, 640
    data_note = "synthetic epochChangeHashData payloads (numpy, host memory), one copy per ack"

    def __init__(self, a, eng, dev, rank):
        from mirbft_amd import SliceArrays, hashdata

        self.a, self.eng = a, eng
        _, n0, _, self.desc = CONFIGS[4]
        self.n = n = a.requests or n0
        self.dedup = bool(a.dedup)
        self.buf, so, sl, self.first, self.origin = hashdata.epoch_change_cycle(
            self.N_NODES, n, self.N_CP, self.N_P, self.N_Q, new_epoch=2 + rank)
        self.sl = SliceArrays.from_buffer(self.buf, so, sl, self.first)
        self.plen = self.buf.size // n
        self.slices_per_req = int(self.first[1])
        self.bytes_hashed = self.buf.size
        self.digests = n
        self.distinct = min(n, self.N_NODES)
        self.hashed_reqs = self.distinct if self.dedup else n
        self.req_blocks = int(blocks(self.plen)) * self.hashed_reqs
        self.plan = None
        eng.set_stream(None)  # host API on the engine's own stream

    def step(self):
        self.eng.hash_slice_arrays(self.sl, dedup=self.dedup)

    def after(self):
        pass

    def dominant(self):
        n_m, ms_m = self.eng.kernel_time(KERNEL_MSGS)
        return "sha256_msgs_kernel", n_m, ms_m, self.req_blocks, self.hashed_reqs * (self.plen + 32)

    def self_check(self):
        import hashlib

        got = self.eng.hash_slice_arrays(self.sl, dedup=self.dedup)
        ok = self.eng.last_unique == self.hashed_reqs
        for r in list(range(0, self.n, max(1, self.n // 16))) + [self.n - 1]:
            want = hashlib.sha256(self.buf[r * self.plen:(r + 1) * self.plen].tobytes()).digest()
            ok &= got[r].tobytes() == want
        return bool(ok)

    def pcie(self):
        # One cycle of the benched form, after a call on every ring slot (the
        # first call on a slot allocates its pinned staging).
        for _ in range(5):
            self.eng.hash_slice_arrays(self.sl, dedup=self.dedup)
        self.host_phases = self.eng.host_profile()
        other = not self.dedup
        reps, t0 = 5, time.perf_counter()
        for _ in range(reps):
            self.eng.hash_slice_arrays(self.sl, dedup=other)
        dt = (time.perf_counter() - t0) / reps
        return {"dedup": other, "digests_per_s": self.n / dt, "ms_per_call": dt * 1e3,
                "note": "the same cycle with dedup toggled (A/B)"}

    def cpu_baseline(self, seconds):
        o = _oracle()
        k = min(self.n, 256)  # 256 x 61.6 KB = 15.8 MB of the same requests
        arena = self.buf[: k * self.plen]
        off = np.arange(k, dtype=np.uint64) * self.plen
        ln = np.full(k, self.plen, dtype=np.uint32)
        res = _time_cpu(lambda t: o.hash_requests(arena, off, ln, threads=t), seconds, (1, pool_threads()))
        done1, dt1 = res[1]
        tp = max(res)
        return {
            "value": done1 * k / dt1, "unit": "digests/s", "cores": 1, "kind": "port",
            "sample": f"{done1} passes x {k} EpochChangeAck requests x {self.plen} B, {dt1:.1f} s, oracle C port "
                      f"of processor.go:133-143 (every ack hashed, as the reference does), SHA-NI compression",
            "pool": {"value": res[tp][0] * k / res[tp][1], "threads": tp},
            "cpu": _cpu_model(),
            **_cpu_facts(),
        }

    def config_fields(self):
        return {"requests_per_gpu": self.n, "payload_bytes": self.plen, "slices_per_request": self.slices_per_req,
                "origins": self.N_NODES, "distinct_payloads": self.distinct, "dedup": self.dedup,
                "input": "host slices (Go-side [][]byte); each step = pack + H2D + kernel + D2H",
                "compressions_per_step_per_gpu": self.req_blocks}

    def extra(self):
        return {"pcie_inclusive_by_design": True, "host_phases_ms": getattr(self, "host_phases", None)}


def small_cycle_bench(a, eng):
    """Config 1 (testengine, 4 nodes x 4 clients x 200 requests, BatchSize 20):
    a Ready() cycle's Actions.Hash is tens of request hashes -- LE64(client) ||
    LE64(reqNo) || data, data = LE64(client) || "-" || LE64(reqNo), 3 slices,
    33 bytes (state_machine.go:313-317, testengine/recorder.go:158-174) --
    plus batch hashes over 20 RequestAck digests (sequence.go:154-157, 20
    slices of 32 B), all independent HashRequests of one call.  Per-call
    latency (median / p90 over `reps` calls) of the synchronous host API
    (mirsha_hash_slices), the asynchronous one (submit + wait) and the one-core
    CPU port of the loop on the same slices."""
    from mirbft_amd import SliceArrays

    o = _oracle()
    reps, rows = 300, []
    for n_req in (16, 80, 320):
        n_bat = max(1, n_req // 20)
        buf = np.zeros(33 * n_req + 32 * 20 * n_bat, dtype=np.uint8)
        so, sl, first = [], [], [0]
        for i in range(n_req):
            c, r = i % 4, i // 4
            b = 33 * i
            buf[b:b + 8] = np.frombuffer(np.uint64(c).tobytes(), np.uint8)
            buf[b + 8:b + 16] = np.frombuffer(np.uint64(r).tobytes(), np.uint8)
            buf[b + 16:b + 24] = buf[b:b + 8]
            buf[b + 24] = ord("-")
            buf[b + 25:b + 33] = buf[b + 8:b + 16]
            so += [b, b + 8, b + 16]
            sl += [8, 8, 17]
            first.append(len(so))
        rng = np.random.default_rng(n_req)
        base = 33 * n_req
        buf[base:] = rng.integers(0, 256, buf.size - base, dtype=np.uint8)
        for k in range(n_bat):
            for j in range(20):
                so.append(base + 32 * (20 * k + j))
                sl.append(32)
            first.append(len(so))
        arrays = SliceArrays.from_buffer(buf, np.array(so, np.uint64), np.array(sl, np.uint64), np.array(first, np.uint32))
        n = arrays.n
        want = o.hash_slices(arrays.ptr, arrays.len, arrays.first)
        got = eng.hash_slice_arrays(arrays)
        assert np.array_equal(got, want), "small-cycle digests differ from the oracle"

        def lat(fn):
            for _ in range(20):
                fn()
            t = np.empty(reps)
            for k in range(reps):
                t0 = time.perf_counter()
                fn()
                t[k] = time.perf_counter() - t0
            return float(np.median(t) * 1e6), float(np.percentile(t, 90) * 1e6)

        out = np.empty((n, 32), np.uint8)
        sync = lat(lambda: eng.hash_slice_arrays(arrays))
        asyn = lat(lambda: eng.wait(eng.submit_slices(arrays)))
        cpu = lat(lambda: o.hash_slices(arrays.ptr, arrays.len, arrays.first, out))
        rows.append({"request_hashes": n_req, "batch_hashes": n_bat, "hash_requests": n,
                     "hash_slices_us": sync[0], "hash_slices_p90_us": sync[1],
                     "submit_wait_us": asyn[0], "submit_wait_p90_us": asyn[1],
                     "cpu_1core_us": cpu[0], "cpu_1core_p90_us": cpu[1]})
    last = rows[-1]
    print(json.dumps({
        "metric": "Ready()-cycle hash latency, small testengine cycles (BASELINE config 1 shape)",
        "value": last["hash_requests"] / (last["hash_slices_us"] * 1e-6), "unit": "digests/s",
        "n_gpus": 1, "steps": reps, "warmup": 20, "ms_per_step": last["hash_slices_us"] / 1e3,
        "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic testengine requests (recorder.go:158-174) + random RequestAck digests",
        "config": {"workload": "config1: tens of 33-B request hashes + BatchSize-20 batch hashes per Ready() cycle, "
                               "host slices through the C-ABI, synchronous and asynchronous"},
        "cycles": rows,
        "note": "per-call wall time from host slices to host digests (PCIe both ways, kernel launch, one sync); "
                "cpu_1core = oracle C port of processor.go:133-143 (SHA-NI) on the same slices",
    }), flush=True)


def config3_leg(a, eng, dev):
    """BASELINE config 3 (2^18 x 4 KB requests + VerifyBatch-500 digests) as a
    leg of the default run, after config 2's timed region and self-check
    (rank 0, N = 1): the fused plan's step (request + VerifyBatch chains in
    one launch, readiness counters), its dominant-kernel time and roofline
    fraction, the overlapped-cycles figure on the same plan, the sequential
    plan's request kernel (the CU-block kernel, 4 waves per SIMD), and a
    self-check against the oracle on a sample.  Data generated on the device
    before any timed region; ~3-5 s."""
    import argparse as _ap

    t_start = time.perf_counter()
    steps = min(a.steps, 20)
    out = {}
    for mode in ("auto", "sequential"):
        a3 = _ap.Namespace(**vars(a))
        a3.config, a3.requests, a3.pipeline, a3.steps, a3.warmup = 3, 0, mode, steps, 3
        wl = BatchWorkload(a3, eng, dev, 0)
        for _ in range(a3.warmup):
            wl.step()
        torch.cuda.synchronize(dev)
        t_pw = time.perf_counter()
        while (time.perf_counter() - t_pw) < 0.15:  # untimed pre-warm at this load
            wl.step()
            torch.cuda.synchronize(dev)
        eng.set_timing_mask([KERNEL_MSGS, KERNEL_FUSED] if mode == "auto" else range(32))
        eng.set_timing(True)
        eng.reset_timing()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            wl.step()
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        eng.set_timing(False)
        wl.after()
        kname, n_k, ms_k, work_blocks, hbm = wl.dominant()
        kms = ms_k / max(n_k, 1)
        tops = work_blocks * OPS_PER_COMPRESSION / (ms_k / steps * 1e-3) / 1e12
        tkey = kernel_source_key(a.variant)
        traffic, _ = lookup_traffic(a.traffic_file, tkey, 3, kname)
        step_tops = (wl.req_blocks + wl.bat_blocks) * OPS_PER_COMPRESSION / (dt / steps) / 1e12
        leg = {"plan": wl.plan.mode_name, "ms_per_step": dt / steps * 1e3,
               "digests_per_s": wl.digests * steps / dt, "kernel": kname, "avg_launch_ms": kms,
               "frac": tops / VALU_PEAK_TOPS, "step_frac": step_tops / VALU_PEAK_TOPS,
               "compressions": work_blocks, "step_compressions": wl.req_blocks + wl.bat_blocks,
               "traffic": traffic, "traffic_key": tkey}
        if wl.plan.mode_name == "fused":
            # right behind the timed steps, the chip still at this load's clock
            # (a self-check first left it idle and cooling: profiles/r04g)
            a3.warmup = 30
            leg["overlap_cycles"] = wl.overlap_cycles()
            leg["frac_note"] = ("frac: request + VerifyBatch compressions over the fused launch's time; step_frac: "
                                "the same over ms_per_step")
        else:
            leg["frac_note"] = ("frac: request compressions over the request kernel's time (the batch chains "
                                "follow); step_frac: request + VerifyBatch compressions over ms_per_step")
            leg["batch_kernel_ms"] = wl.batch_ms() / steps
        eng.set_timing_mask(range(32))
        leg["self_check"] = wl.self_check()
        out[wl.plan.mode_name] = leg
        if wl.plan is not None:
            wl.plan.close()
        del wl
        torch.cuda.empty_cache()
    out["workload"] = f"config3: {CONFIGS[3][3]}"
    out["steps"] = steps
    out["leg_seconds"] = time.perf_counter() - t_start
    return out


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def count_devices():
    """Visible GPUs, counted in a throwaway child process: this launching
    parent never imports torch and never initialises the HIP runtime (on ROCm
    torch.cuda.device_count() falls back to hipGetDeviceCount when amdsmi is
    absent, which would start the runtime in the process that forks the
    ranks).  0 when the child fails (no GPU, no torch)."""
    if os.environ.get("MIRSHA_BENCH_COUNT_STUB"):  # CPU tests: the count the child would print
        return int(os.environ["MIRSHA_BENCH_COUNT_STUB"])
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(r.stdout.split()[-1]) if r.returncode == 0 else 0
    except (IndexError, ValueError):
        return 0


def launch_ranks(a):
    """`--gpus N` without a launcher: start N rank processes of this script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on 127.0.0.1),
    forward rank 0's stdout, and return non-zero if any rank fails (the others
    are then stopped by PID).  The parent only counts devices, in a child
    process (count_devices), and never execs: the ranks are children."""
    n = a.gpus
    rehearsal = bool(os.environ.get("MIRSHA_BENCH_DEVICE"))
    if not rehearsal and not a.launch_check:
        vis = count_devices()
        if vis < n:
            print(f"bench.py: --gpus {n} but {vis} device(s) visible (set MIRSHA_BENCH_DEVICE=<d> to rehearse "
                  f"{n} ranks on one device)", file=sys.stderr, flush=True)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, text=True))

    def forward(stream):
        for line in stream:
            sys.stdout.write(line)
            sys.stdout.flush()

    fw = threading.Thread(target=forward, args=(procs[0].stdout,), daemon=True)
    fw.start()

    def stop(signum, _frame):  # a launcher's time limit: take the ranks down with us
        for q in procs:
            if q.poll() is None:
                q.terminate()
        sys.exit(128 + signum)

    import signal

    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    rc = 0
    live = list(range(n))
    while live:
        for r in list(live):
            code = procs[r].poll()
            if code is None:
                continue
            live.remove(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"bench.py: rank {r} exited with {code}; stopping the other ranks", file=sys.stderr, flush=True)
                for q in live:
                    procs[q].terminate()
                deadline = time.time() + 30
                for q in live:
                    try:
                        procs[q].wait(timeout=max(deadline - time.time(), 0.1))
                    except subprocess.TimeoutExpired:
                        procs[q].kill()
        time.sleep(0.05)
    fw.join(timeout=10)
    return rc


def device_identity_check(per_rank, rehearsal):
    """Whether the ranks ran on distinct GPUs, from the device UUIDs (else the
    PCI bus ids) they report.  distinct: True / False, or None when the
    identities are missing, or when MIRSHA_BENCH_DEVICE deliberately puts
    every rank on one device (a rehearsal: not checked)."""
    ids = []
    for p in per_rank:
        u = p.get("device_uuid") or ""
        ids.append(u if u.strip("0-") else (str(p.get("pci_bus_id")) if p.get("pci_bus_id") is not None else None))
    if len(per_rank) < 2:
        return {"distinct": True, "note": "one rank"}
    if rehearsal:
        return {"distinct": None, "note": "rehearsal: every rank on device MIRSHA_BENCH_DEVICE, not checked"}
    if any(i is None for i in ids):
        return {"distinct": None, "note": "device identities unavailable"}
    d = len(set(ids)) == len(ids)
    return {"distinct": d, "note": f"{len(set(ids))} distinct device identities over {len(ids)} ranks"}


def launch_check(a, world, rank):
    """--launch-check: the N>1 plumbing without a device (CPU tests): gloo
    rendezvous, barrier, each rank's request range (BatchWorkload's weak
    scaling: rank r hashes [r n, (r + 1) n)), gather, rank 0's line."""
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    if os.environ.get("MIRSHA_BENCH_CHECK_SLEEP"):  # test hook: ranks that outlive a launcher's signal
        time.sleep(float(os.environ["MIRSHA_BENCH_CHECK_SLEEP"]))
    n = a.requests or CONFIGS[a.config if a.config in CONFIGS else 2][1]
    # The per-rank self-check path on the CPU: this rank's range (at most 4,096
    # requests of config 2's shape) hashed by the oracle stands in for the
    # device digests; a test hook corrupts the final (partial) batch digest of
    # one rank, which the AND over ranks must report.
    from mirbft_amd import sharding as _sh

    m = min(n, 4096)
    data_len, bs = CONFIGS[2][0], CONFIGS[2][2]
    seed, first_req = SEED_BASE + 2, rank * n
    o = _oracle()
    idx, first = _sh.batch_lists(m, bs)
    req = o.hash_requests(o.gen_requests(seed, first_req, m, data_len), np.arange(m, dtype=np.uint64) * (16 + data_len),
                          np.full(m, 16 + data_len))
    bat = o.batch_digests(req, idx, first)
    if os.environ.get("MIRSHA_BENCH_CHECK_CORRUPT_RANK") == str(rank):
        bat[-1, 0] ^= 1
    ok = check_batch_windows(seed, first_req, data_len, idx, first, req, bat)
    info = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "pid": os.getpid(),
            "first_request": rank * n, "requests": n, "self_check": ok, "device_uuid": f"launch-check-{rank}"}
    per_rank = [info]
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, info)
    if rank == 0:
        print(json.dumps({"metric": "SHA-256 digests/s (request + batch digests), Actions.Hash stream",
                          "value": None, "unit": "digests/s", "n_gpus": world, "steps": a.steps,
                          "warmup": a.warmup, "launch_check": True, "per_rank": per_rank,
                          "self_check": all(p["self_check"] for p in per_rank),
                          "distributed": {"backend": "gloo" if world > 1 else None,
                                          "device_identity": device_identity_check(per_rank, False)},
                          "note": "launcher plumbing only: no device; self_check = the oracle's own digests of "
                                  "each rank's range through the per-rank window check"}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    a = parse()
    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher's WORLD_SIZE is {world}")
    if a.launch_check:
        launch_check(a, world, rank)
        return
    _import_product()
    # Rehearsal knob for the N>1 path on a one-GPU box (never set by the
    # driver): every rank on device MIRSHA_BENCH_DEVICE.  The control plane
    # (barriers, max / sum of timings, the per-rank gather) is gloo at any N:
    # the data path has no collective (north_star), so RCCL would carry only
    # these few host scalars, and gloo is the branch every rehearsal ran.
    # MIRSHA_BENCH_DIST_BACKEND=nccl is an A/B knob.
    rehearsal = bool(os.environ.get("MIRSHA_BENCH_DEVICE"))
    if rehearsal:
        local = int(os.environ["MIRSHA_BENCH_DEVICE"])
    backend = os.environ.get("MIRSHA_BENCH_DIST_BACKEND", "gloo")
    dist = None
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist

        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    # reductions live on the device for RCCL, on the host for gloo
    red_dev = dev if backend == "nccl" else torch.device("cpu")

    eng = Engine(local)
    eng.set_variant(a.variant)
    if a.config == 1:  # latency of small host-API cycles (own JSON line)
        small_cycle_bench(a, eng)
        return
    stream = torch.cuda.current_stream(dev)
    eng.set_stream(stream.cuda_stream)

    if a.config == 5:
        wl = MixedWorkload(a, eng, dev, rank, world)
    else:
        wl = {4: EpochChangeWorkload}.get(a.config, BatchWorkload)(a, eng, dev, rank)
    torch.cuda.synchronize(dev)

    # PCIe-inclusive host-API rate (rank 0, N=1 only), measured before the
    # device-resident steps.
    pcie = wl.pcie() if rank == 0 and world == 1 and not a.no_pcie else None
    cgo = wl.cgo_path() if rank == 0 and world == 1 and not a.no_pcie and hasattr(wl, "cgo_path") else None
    multi = None
    if rank == 0 and world == 1 and not a.no_pcie and a.config == 2 and hasattr(wl, "multi_device"):
        try:  # an extra leg: a failure is reported in the line, not fatal to it
            multi = wl.multi_device()
        except Exception as e:  # noqa: BLE001
            multi = {"error": f"{type(e).__name__}: {e}"}
    torch.cuda.synchronize(dev)

    for _ in range(a.warmup):
        wl.step()
    torch.cuda.synchronize(dev)
    # Untimed pre-warm: the same steps until prewarm_ms of wall time have
    # passed, so the timed region starts at the clock the chip holds under
    # this load (DVFS; MI355X_MICROARCH.md).  Reported in the JSON line.
    prewarm_steps, t_pw = 0, time.perf_counter()
    while a.prewarm_ms > 0 and (time.perf_counter() - t_pw) * 1e3 < a.prewarm_ms:
        for _ in range(8):
            wl.step()
        prewarm_steps += 8
        torch.cuda.synchronize(dev)
    prewarm_ms = (time.perf_counter() - t_pw) * 1e3
    if dist:
        dist.barrier()

    def timed(with_events, every=1):
        eng.set_timing(with_events)
        eng.reset_timing()
        sampled = set(event_steps(a.steps, every))
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(a.steps):
            if with_events and every > 1:
                eng.set_timing(i in sampled)  # event_steps: every k-th, never the first
            wl.step()
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        el = time.perf_counter() - t0
        eng.set_timing(False)
        return el

    if a.timed_kernels == "dominant":
        eng.set_timing_mask([KERNEL_MSGS, KERNEL_FUSED, KERNEL_OVERLAP])
    every = max(1, min(a.event_every, a.steps)) if a.events_in_timed_loop else 1
    dt = timed(bool(a.events_in_timed_loop), every)
    ev_steps = len(event_steps(a.steps, every))  # steps whose dominant launches carry events
    if not a.events_in_timed_loop:
        timed(True)
    wl.after()
    kname, n_k, ms_k, work_blocks, hbm_bytes = wl.dominant()
    if a.timed_kernels == "dominant":
        # Second-pass timing of the other kernels (batch kernel figures in the
        # line's extras); the value and the roofline come from the pass above.
        eng.set_timing_mask(range(32))
        timed(True)
    # Batch-pass kernel time of the last timing pass, read before
    # overlap_cycles() resets the engine's timers.
    if hasattr(wl, "batch_ms"):
        wl.batch_ms_timed = wl.batch_ms()
    # SURVEY.md §8d asks for a median over repeats: the same timed region
    # --repeat-regions more times, bare (no events), each bracketed like the
    # headline's; reported beside the value, never as it.
    rep_ms = [timed(False) / a.steps * 1e3 for _ in range(max(0, a.repeat_regions))]

    # Configs 2/3 with a sequential plan: the overlapped-cycles figure, right
    # behind the timed region too (the chip still at its load clock).
    if rank == 0 and a.overlap_extra and hasattr(wl, "overlap_cycles"):
        wl.ovl = wl.overlap_cycles()

    # Clock probe right behind the timed region (chip still at its load clock):
    # register-only compressions in the request kernel's round form.
    probe = None
    if a.probe_iters > 0:
        ghz, cyc = eng.clock_probe(a.probe_iters)
        probe = {"clock_ghz": ghz, "cycles_per_wave_compression": cyc}

    dt_rank = dt
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # Every rank checks the last step of its OWN request range against the CPU
    # oracle on samples (first / last / random requests and the batches over
    # them, the final partial batch included); the line's self_check is the
    # AND over ranks, each rank's own is in per_rank.
    check_ok = bool(wl.self_check())

    # Whole-job totals: the sum over ranks (config 5's block-balanced shards
    # differ in request count per rank).  step_compressions = every
    # compression of a step (request + batch digests), BASELINE.md's per-config
    # accounting, for roofline.step_frac.
    step_comp = int(wl.req_blocks) + int(getattr(wl, "bat_blocks", 0))
    tot = torch.tensor([float(wl.digests), float(wl.bytes_hashed), float(step_comp)], dtype=torch.float64,
                       device=red_dev)
    if dist:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    value = float(tot[0].item()) * a.steps / dt
    gbps = float(tot[1].item()) * a.steps / dt / 1e9
    ms_per_step_k = ms_k / ev_steps  # all launches of the dominant kernel in one (sampled) step
    achieved_tops = work_blocks * OPS_PER_COMPRESSION / (ms_per_step_k * 1e-3) / 1e12
    hbm_gbs = hbm_bytes / (ms_per_step_k * 1e-3) / 1e9
    # per-GPU average over the whole step's wall time (max over ranks)
    step_tops = float(tot[2].item()) / world * OPS_PER_COMPRESSION / (dt / a.steps) / 1e12

    tkey = kernel_source_key(a.variant)
    traffic, tentry = lookup_traffic(a.traffic_file, tkey, a.config, kname)
    # Measured ceiling: the probe's register-only compression rate on this box
    # (1,024 SIMDs x 64 lanes per wave-compression) and the clock it ran at.
    measured = None
    if probe and probe["cycles_per_wave_compression"] > 0:
        ceil_cps = 1024 * 64 * probe["clock_ghz"] * 1e9 / probe["cycles_per_wave_compression"]
        achieved_cps = work_blocks / (ms_per_step_k * 1e-3)
        measured = {"compressions_per_s": ceil_cps, "frac": achieved_cps / ceil_cps,
                    "cycles_per_wave_compression": probe["cycles_per_wave_compression"],
                    "spec_cycles_per_wave_compression": 2 * OPS_PER_COMPRESSION,
                    "note": "clock probe: 8 waves/SIMD of register-only compressions (the request kernel's "
                            "round form), right after the timed region"}

    # Config 3 (the north_star's 4 KB target) as a leg of the default run.
    c3 = None
    if rank == 0 and world == 1 and a.config == 2 and a.config3_leg and a.requests == 0:
        eng.set_stream(stream.cuda_stream)
        c3 = config3_leg(a, eng, dev)

    cpu = wl.cpu_baseline(a.cpu_seconds) if rank == 0 and world == 1 and a.cpu_seconds > 0 else None

    # Per-rank evidence (control plane, after the timed region): which device
    # each rank ran on and its own dominant-kernel time, so a multi-GPU line
    # shows N distinct GPUs each near the single-GPU kernel rate.
    props = torch.cuda.get_device_properties(dev)
    rank_info = {"rank": rank, "local_rank": local, "device": local,
                 "device_uuid": str(getattr(props, "uuid", "")), "pci_bus_id": getattr(props, "pci_bus_id", None),
                 "digests": int(wl.digests), "compressions": int(work_blocks),
                 "first_request": int(getattr(wl, "first_req", 0)), "wall_ms_per_step": dt_rank / a.steps * 1e3,
                 "kernel": kname, "kernel_avg_launch_ms": ms_k / max(n_k, 1),
                 "frac": achieved_tops / VALU_PEAK_TOPS, "self_check": check_ok}
    per_rank = [rank_info]
    if dist:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, rank_info)
    check_all = all(p["self_check"] for p in per_rank)
    ident = device_identity_check(per_rank, rehearsal)
    if ident["distinct"] is False:
        raise SystemExit(f"bench.py: rank {rank}: ranks share a device ({ident['note']}); a multi-GPU line "
                         f"needs one GPU per rank (MIRSHA_BENCH_DEVICE rehearses on one device)")

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
            "data": getattr(wl, "data_note", "synthetic (splitmix64 request stream generated on device, SURVEY.md §8d)"),
            "config": {
                "workload": f"config{a.config}: {wl.desc}",
                **wl.config_fields(),
                "parallelism": f"request-range shards x{world}, no collective",
                "kernel_variant": {0: "lds", 1: "direct", 4: "lowocc", 5: "lds_only", 6: "pair", 10: "cu"}[a.variant],
            },
            "gb_per_s_hashed": gbps,
            "roofline": {
                "bound": "valu",
                "achieved": achieved_tops,
                "peak": VALU_PEAK_TOPS,
                "unit": "TOP/s",
                "frac": achieved_tops / VALU_PEAK_TOPS,
                "step_frac": step_tops / VALU_PEAK_TOPS,
                "step_achieved": step_tops,
                "step_compressions_per_gpu": float(tot[2].item()) / world,
                "frac_note": "frac = the dominant kernel's compressions over its own HIP-event time (events bound "
                             "to the kernel's dispatches, timed_launches of the timed region: every event_every-th "
                             "step); step_frac = every compression of a step (request + batch digests, "
                             "BASELINE.md's accounting) over ms_per_step, per GPU",
                "traffic": traffic,
                "kernel": kname,
                "avg_launch_ms": ms_k / max(n_k, 1),
                "launches_per_step": n_k / ev_steps,
                "timed_launches": n_k,
                "kernel_ms_per_step": ms_per_step_k,
                "work": f"{work_blocks} compressions x {OPS_PER_COMPRESSION} int32 ops per step "
                        f"(over {n_k // ev_steps} launch(es))",
                "hbm_algorithmic_gb_per_s": hbm_gbs,
                "hbm_frac": hbm_gbs / HBM_PEAK_GBS,
                "traffic_key": tkey,
                "traffic_source": (tentry or {}).get("source"),
                "traffic_over_algorithmic": (traffic / hbm_bytes) if traffic else None,
                "measured_peak": measured,
                "note": "SHA-256 is int32 VALU work (no MFMA shape); hbm/mfma bounds do not apply; "
                        "traffic = PMC HBM bytes per launch of this exact kernel source (null if not profiled)",
            },
            "prewarm_ms": prewarm_ms,
            "prewarm_steps": prewarm_steps,
            "effective_clock_ghz": probe["clock_ghz"] if probe else None,
            **wl.extra(),
            "events_in_timed_loop": bool(a.events_in_timed_loop),
            "event_every": every,
            "repeat_regions": ({"ms_per_step": rep_ms, "median_ms_per_step": float(np.median(rep_ms)),
                                "note": "the same timed region again, bare, max over ranks not taken; the value "
                                        "is the first region's"} if rep_ms else None),
            "timed_kernels": a.timed_kernels,
            "self_check": check_all,
            "self_check_scope": "every rank: its own range's first and last batch-aligned windows (the final "
                                "partial batch included) and 4 random ones, request + batch digests vs the oracle",
            "per_rank": per_rank,
            "distributed": {"world_size": world, "backend": backend if dist else None,
                            "device_identity": ident,
                            "data_path_collectives": "none: each rank hashes its own request range; "
                                                     "barriers and max / sum reductions of timings only"},
            "pcie_inclusive": pcie,
            "multi_device": multi,
            "cgo_path": cgo,
            "config3": c3,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
