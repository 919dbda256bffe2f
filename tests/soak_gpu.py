#!/usr/bin/env python3
"""Randomised GPU soak (run by hand / tools/gpu scripts, not collected by
pytest): for a time budget, random shapes through every entry point --
host arenas with gaps and odd alignments, sliced requests with duplicates
(plain and dedup), async submit / wait in shuffled order, request -> list
digests (nulls, empty and shared lists) through the host call and through
device plans in every mode, tile-queue count and list-tile form, overlapped
cycles, launches of 65K-400K requests, fused plans with split tiles,
checkpoint chains, arena submissions in random chunks (mirsha_submit_batch
and its multi-device twin, page-locked or pageable arenas and outputs) -- each checked bit for bit against the oracle (test infrastructure,
oracle/).  Prints a progress line every ~15 s; exits 1 at the first mismatch
with the seed that reproduces it.

Usage: python tests/soak_gpu.py [--seconds 120] [--seed 1]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import oracle_py  # noqa: E402
from mirbft_amd import Engine  # noqa: E402
from mirbft_amd import _lib  # noqa: E402
from mirbft_amd import sharding  # noqa: E402

EDGE = [0, 1, 15, 16, 17, 55, 56, 63, 64, 65, 119, 120, 127, 128, 183, 184, 247, 248, 272, 4112]


def lengths(rng, n):
    kind = rng.integers(0, 4)
    if kind == 0:  # one length (uniform tiles, tail form)
        return np.full(n, int(rng.choice(EDGE + [int(rng.integers(0, 400))])), dtype=np.uint32)
    if kind == 1:  # block-boundary mix
        return rng.choice(EDGE, n).astype(np.uint32)
    if kind == 2:  # small uniform random
        return rng.integers(0, 600, n).astype(np.uint32)
    ln = rng.integers(0, 300, n).astype(np.uint32)  # a few long messages
    ln[rng.random(n) < 0.01] = rng.integers(1000, 70000)
    return ln


def arena_for(rng, ln):
    """Messages at random gaps (some overlapping) from a random base alignment."""
    n = ln.size
    gaps = rng.integers(0, 9, n).astype(np.uint64) if rng.random() < 0.5 else np.zeros(n, np.uint64)
    off = np.zeros(n, dtype=np.uint64)
    pos = np.uint64(rng.integers(0, 4))
    for i in range(n):
        off[i] = pos
        pos += np.uint64(ln[i]) + gaps[i]
        if rng.random() < 0.02 and ln[i] > 8:  # overlap the next message with this one
            pos -= np.uint64(4)
    end = int((off + ln.astype(np.uint64)).max()) if n else 0
    arena = rng.integers(0, 256, max(end, int(pos)) + 1, dtype=np.uint8)
    return arena, off


def lists_for(rng, n, n_lists):
    sizes = rng.integers(0, int(rng.choice([4, 21, 60, 501])), n_lists)
    sizes[rng.random(n_lists) < 0.1] = 0
    idx = rng.integers(0, max(n, 1), int(sizes.sum())).astype(np.uint32)
    idx[rng.random(idx.size) < 0.05] = _lib.MIRSHA_NULL_INDEX
    first = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    return idx, first


def check(ok, what, seed):
    if not ok:
        raise AssertionError(f"MISMATCH: {what} (seed {seed})")


def case_host(eng, rng, seed):
    n = int(rng.integers(1, 6000))
    ln = lengths(rng, n)
    arena, off = arena_for(rng, ln)
    want = oracle_py.hash_requests(arena, off, ln)
    check(np.array_equal(eng.hash_batch(arena, off, ln), want), f"hash_batch n={n}", seed)
    idx, first = lists_for(rng, n, int(rng.integers(0, 400)))
    req, bat = eng.hash_requests_then_batches(arena, off, ln, idx, first)
    check(np.array_equal(req, want), "requests_then_batches: requests", seed)
    check(np.array_equal(bat, oracle_py.batch_digests(want, idx, first)), "requests_then_batches: lists", seed)


def case_slices(eng, rng, seed):
    n = int(rng.integers(1, 800))
    pool = [rng.integers(0, 256, int(x), dtype=np.uint8).tobytes() for x in lengths(rng, max(n // 4, 1))]
    reqs = []
    for _ in range(n):
        b = pool[int(rng.integers(0, len(pool)))]
        cuts = sorted(int(x) for x in rng.integers(0, len(b) + 1, int(rng.integers(0, 6))))
        parts, last = [], 0
        for c in cuts + [len(b)]:
            parts.append(b[last:c])
            last = c
        reqs.append(parts)
    want = oracle_py.hash_messages([b"".join(r) for r in reqs])
    dedup = bool(rng.random() < 0.5)
    check(np.array_equal(eng.hash_slices(reqs, dedup=dedup), want), f"hash_slices dedup={dedup} n={n}", seed)
    # async: several submissions, waited in a shuffled order
    batches = [reqs[i::3] for i in range(3)]
    tickets = [eng.submit_slices(b, dedup=bool(rng.random() < 0.5)) for b in batches]
    for k in rng.permutation(3):
        got = eng.wait(tickets[k])
        check(np.array_equal(got, want[k::3]), "submit/wait", seed)


def case_plan(eng, rng, seed):
    n = int(rng.integers(1, 20000))
    ln = lengths(rng, n)
    ln = np.minimum(ln, 5000).astype(np.uint32)
    arena, off = arena_for(rng, ln)
    idx, first = lists_for(rng, n, int(rng.integers(1, 1500)))
    mode = str(rng.choice(["auto", "fused", "sequential"]))
    os.environ["MIRSHA_AB"] = "1"  # schedule knobs below are read only with MIRSHA_AB=1
    os.environ["MIRSHA_FUSED_PACE"] = str(int(rng.integers(1, 5)))
    os.environ["MIRSHA_FUSED_LIST_TILES"] = str(int(rng.integers(0, 3)))
    plan = eng.pipeline(n, idx, first, ln, mode=mode)
    os.environ.pop("MIRSHA_FUSED_PACE")
    os.environ.pop("MIRSHA_FUSED_LIST_TILES")
    os.environ.pop("MIRSHA_AB")
    want = oracle_py.hash_requests(arena, off, ln)
    want_l = oracle_py.batch_digests(want, idx, first)
    d_arena = torch.from_numpy(arena).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.from_numpy(ln.view(np.int32)).cuda()
    nl = first.size - 1
    d_req = [torch.zeros((n, 32), dtype=torch.uint8, device="cuda") for _ in range(2)]
    d_lst = torch.zeros((max(nl, 1), 32), dtype=torch.uint8, device="cuda")
    args = (d_arena.data_ptr(), arena.size, d_off.data_ptr(), d_len.data_ptr())
    for _ in range(int(rng.integers(1, 4))):
        d_req[0].zero_()
        d_lst.zero_()
        torch.cuda.synchronize()  # torch's stream vs the engine's own (non-blocking) stream
        eng.hash_requests_then_batches_device(plan, *args, d_req[0].data_ptr(), d_lst.data_ptr())
        plan.status()
        check(np.array_equal(d_req[0].cpu().numpy(), want), f"plan {mode}: requests n={n}", seed)
        check(np.array_equal(d_lst.cpu().numpy()[:nl], want_l), f"plan {mode}: lists ({nl})", seed)
    if plan.mode_name in ("fused", "sequential") and rng.random() < 0.5:  # overlapped cycles + flush
        for i in range(3):
            prev = d_req[(i + 1) % 2].data_ptr() if i else 0
            d_lst.zero_()
            torch.cuda.synchronize()
            if i < 2:
                eng.pipeline_overlap_device(plan, *args, d_req[i % 2].data_ptr(), prev, d_lst.data_ptr())
            else:
                eng.pipeline_overlap_device(plan, 0, 0, 0, 0, 0, prev, d_lst.data_ptr())
            eng.sync()
            if i < 2:
                check(np.array_equal(d_req[i % 2].cpu().numpy(), want), f"overlap {mode}: requests", seed)
            if i:
                check(np.array_equal(d_lst.cpu().numpy()[:nl], want_l), f"overlap {mode}: lists", seed)
        plan.status()
    plan.close()


def case_large(eng, rng, seed):
    """Launches past 1,024 tiles (the LDS request kernel at full occupancy,
    the uniform-tile and tail forms, bucketed orders) on device buffers."""
    n = int(rng.integers(65_537, 400_000))
    kind = rng.integers(0, 3)
    if kind == 0:
        ln = np.full(n, int(rng.choice(EDGE[1:] + [int(rng.integers(1, 700))])), dtype=np.uint32)
    elif kind == 1:
        ln = rng.choice(EDGE, n).astype(np.uint32)
    else:
        ln = rng.integers(0, 700, n).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(ln[:-1].astype(np.uint64), out=off[1:])
    off += np.uint64(rng.integers(0, 4))
    arena = rng.integers(0, 256, int(off[-1]) + int(ln[-1]) + 1, dtype=np.uint8)
    want = oracle_py.hash_requests(arena, off, ln, threads=8)
    d_arena = torch.from_numpy(arena).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.from_numpy(ln.view(np.int32)).cuda()
    d_out = torch.zeros((n, 32), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    eng.hash_batch_device(d_arena.data_ptr(), arena.size, d_off.data_ptr(), d_len.data_ptr(), None, n,
                          d_out.data_ptr())
    eng.sync()
    check(np.array_equal(d_out.cpu().numpy(), want), f"large hash_batch_device n={n} kind={kind}", seed)
    if rng.integers(0, 2):
        # BatchSize lists over consecutive requests (sequence.go:154-157), more
        # than 32,768 of them: the sequential plan's chain kernel, identity lists
        # in its computed-index form (constant padding block for even sizes),
        # a permuted near miss in the loaded form
        bs = int(rng.integers(1, n // 32_769 + 1))
        idx, first = sharding.batch_lists(n, bs)
        if rng.integers(0, 4) == 0:
            idx = rng.permutation(n).astype(np.uint32)
    else:
        idx, first = lists_for(rng, n, int(rng.integers(1, 3000)))
    plan = eng.pipeline(n, idx, first, ln, mode=str(rng.choice(["auto", "fused", "sequential"])))
    d_lst = torch.zeros((first.size - 1, 32), dtype=torch.uint8, device="cuda")
    d_out.zero_()
    torch.cuda.synchronize()
    eng.hash_requests_then_batches_device(plan, d_arena.data_ptr(), arena.size, d_off.data_ptr(), d_len.data_ptr(),
                                          d_out.data_ptr(), d_lst.data_ptr())
    plan.status()
    check(np.array_equal(d_out.cpu().numpy(), want), f"large plan {plan.mode_name}: requests n={n}", seed)
    check(np.array_equal(d_lst.cpu().numpy(), oracle_py.batch_digests(want, idx, first)),
          f"large plan {plan.mode_name}: lists", seed)
    plan.close()


def case_split(eng, rng, seed):
    """Fused plans with more tiles than tile-wave slots (split tiles run as
    block-range segments, FusedArgs::n_split): 1-4 tile queues, a few to a
    few hundred tiles over capacity, mixed lengths, shared / null list
    entries; ordinary runs, then overlapped cycles and the flush."""
    pace = int(rng.integers(1, 5))
    n_tiles = pace * 1006 + int(rng.integers(1, 400))
    n = 64 * n_tiles - int(rng.integers(0, 64))
    ln = rng.integers(int(rng.integers(0, 300)), 1300, n).astype(np.uint32)
    arena, off = arena_for(rng, ln)
    idx, first = lists_for(rng, n, int(rng.integers(200, 3000)))
    os.environ["MIRSHA_AB"] = "1"
    os.environ["MIRSHA_FUSED_PACE"] = str(pace)
    plan = eng.pipeline(n, idx, first, ln, mode="fused")
    os.environ.pop("MIRSHA_FUSED_PACE")
    os.environ.pop("MIRSHA_AB")
    want = oracle_py.hash_requests(arena, off, ln, threads=8)
    want_l = oracle_py.batch_digests(want, idx, first)
    d_arena = torch.from_numpy(arena).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.from_numpy(ln.view(np.int32)).cuda()
    nl = first.size - 1
    d_req = [torch.zeros((n, 32), dtype=torch.uint8, device="cuda") for _ in range(2)]
    d_lst = torch.zeros((max(nl, 1), 32), dtype=torch.uint8, device="cuda")
    args = (d_arena.data_ptr(), arena.size, d_off.data_ptr(), d_len.data_ptr())
    tag = f"split pace={pace} tiles={n_tiles} split={plan.split_tiles()}"
    for _ in range(2):
        d_req[0].zero_()
        d_lst.zero_()
        torch.cuda.synchronize()
        eng.hash_requests_then_batches_device(plan, *args, d_req[0].data_ptr(), d_lst.data_ptr())
        plan.status()
        check(np.array_equal(d_req[0].cpu().numpy(), want), tag + ": requests", seed)
        check(np.array_equal(d_lst.cpu().numpy()[:nl], want_l), tag + ": lists", seed)
    # a run whose lengths differ from the plan's (prefixes of the planned
    # messages: split-tile segments past a tile's end are skipped), then the
    # planned lengths again on the same plan
    short = (ln // int(rng.integers(2, 6))).astype(np.uint32)
    want_s = oracle_py.hash_requests(arena, off, short, threads=8)
    d_len_s = torch.from_numpy(short.view(np.int32)).cuda()
    d_req[1].zero_()
    d_lst.zero_()
    torch.cuda.synchronize()
    eng.hash_requests_then_batches_device(plan, d_arena.data_ptr(), arena.size, d_off.data_ptr(), d_len_s.data_ptr(),
                                          d_req[1].data_ptr(), d_lst.data_ptr())
    plan.status()
    check(np.array_equal(d_req[1].cpu().numpy(), want_s), tag + ": short-run requests", seed)
    check(np.array_equal(d_lst.cpu().numpy()[:nl], oracle_py.batch_digests(want_s, idx, first)),
          tag + ": short-run lists", seed)
    for i in range(3):
        prev = d_req[(i + 1) % 2].data_ptr() if i else 0
        d_lst.zero_()
        torch.cuda.synchronize()
        if i < 2:
            eng.pipeline_overlap_device(plan, *args, d_req[i % 2].data_ptr(), prev, d_lst.data_ptr())
        else:
            eng.pipeline_overlap_device(plan, 0, 0, 0, 0, 0, prev, d_lst.data_ptr())
        eng.sync()
        if i < 2:
            check(np.array_equal(d_req[i % 2].cpu().numpy(), want), tag + ": overlap requests", seed)
        if i:
            check(np.array_equal(d_lst.cpu().numpy()[:nl], want_l), tag + ": overlap lists", seed)
    plan.status()
    plan.close()


def case_chains(eng, rng, seed):
    """Streaming checkpoint chains (mirsha_chains_*) against hashlib streaming
    hashers: uniform and skewed writes (one chain taking most digests), sums of
    repeated / random ids, resets."""
    import hashlib

    from mirbft_amd import CheckpointChains

    n = int(rng.integers(1, 3000))
    ch = CheckpointChains(eng, n)
    ref = [hashlib.sha256() for _ in range(n)]
    for cycle in range(int(rng.integers(1, 8))):
        m = int(rng.integers(0, 5000))
        digests = rng.integers(0, 256, (m, 32), dtype=np.uint8)
        if rng.random() < 0.3:  # skewed: one hot chain
            chain_of = np.where(rng.random(m) < 0.9, int(rng.integers(0, n)), rng.integers(0, n, m)).astype(np.uint32)
        else:
            chain_of = rng.integers(0, n, m).astype(np.uint32)
        ch.write(digests, chain_of)
        for d, c in zip(digests, chain_of):
            ref[c].update(d.tobytes())
        cp = rng.integers(0, n, int(rng.integers(0, 40))).astype(np.uint32)
        got = ch.sum(cp)
        check([g.tobytes() for g in got] == [ref[c].digest() for c in cp], f"chains n={n} cycle {cycle}", seed)
        if rng.random() < 0.5:
            cp = np.unique(cp)
            ch.reset(cp)
            for c in cp:
                ref[c] = hashlib.sha256()
    ch.close()


def case_multi(multi, rng, seed):
    """The multi-device drop-in (two contexts on device 0): slices with empty
    requests and empty slices, sync and async (with and without dedup)."""
    from mirbft_amd import SliceArrays

    n = int(rng.integers(1, 30000))
    ln = lengths(rng, n)
    arena, off = arena_for(rng, ln)
    base = arena.ctypes.data
    # 1-3 slices per request, cut at random points inside each message
    k = rng.integers(1, 4, n)
    ptr, sl, first = [], [], [0]
    for i in range(n):
        cuts = np.sort(rng.integers(0, int(ln[i]) + 1, int(k[i]) - 1)) if k[i] > 1 else np.zeros(0, np.int64)
        bounds = [0] + [int(c) for c in cuts] + [int(ln[i])]
        for a, b in zip(bounds, bounds[1:]):
            ptr.append(base + int(off[i]) + a)
            sl.append(b - a)
        first.append(len(ptr))
    arrays = SliceArrays(np.array(ptr, np.uint64), np.array(sl, np.uint64), np.array(first, np.uint32), keep=(arena,))
    want = oracle_py.hash_requests(arena, off, ln, threads=8)
    if rng.random() < 0.5:
        check(np.array_equal(multi.hash_slice_arrays(arrays), want), f"multi sync n={n}", seed)
    else:
        t = multi.submit_slices(arrays, dedup=bool(rng.random() < 0.5))
        check(np.array_equal(multi.wait(t), want), f"multi async n={n}", seed)


def case_arena(eng, multi, pinned, rng, seed):
    """mirsha_submit_batch / mirsha_submit_arena_multi: one cycle's arena (gaps,
    overlaps, odd base) submitted in random chunks, page-locked or pageable
    arena and digest buffer, sometimes a slice submission in between."""
    n = int(rng.integers(1, 20000))
    ln = lengths(rng, n)
    arena, off = arena_for(rng, ln)
    want = oracle_py.hash_requests(arena, off, ln, threads=8)
    p_arena, p_out = pinned
    if rng.random() < 0.5 and arena.size <= p_arena.size:
        a = p_arena[: arena.size]
        a[:] = arena
    else:
        a = arena
    out = p_out[: 32 * n].reshape(n, 32) if rng.random() < 0.5 and 32 * n <= p_out.size else np.empty((n, 32), np.uint8)
    out[:] = 0
    use_multi = rng.random() < 0.3
    e = multi if use_multi else eng
    submit = e.submit_arena if use_multi else e.submit_batch
    cuts = np.unique(np.concatenate([[0, n], rng.integers(0, n + 1, int(rng.integers(0, 12)))]))
    tickets, extra = [], None
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        tickets.append(submit(a, off[lo:hi], ln[lo:hi], out=out[lo:hi]))
        if not use_multi and extra is None and rng.random() < 0.2:
            extra = (lo, hi, eng.submit_slices([[arena[int(o):int(o) + int(m)].tobytes()]
                                                for o, m in zip(off[lo:hi], ln[lo:hi])]))
    if tickets:
        e.wait(tickets[int(rng.integers(0, len(tickets)))])
        e.wait(tickets[-1])
    check(np.array_equal(out, want), f"submit_arena multi={use_multi} n={n} chunks={len(tickets)}", seed)
    if extra is not None:
        lo, hi, t = extra
        check(np.array_equal(eng.wait(t), want[lo:hi]), "slice submission between arena chunks", seed)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120.0)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    from mirbft_amd import MultiEngine

    eng = Engine(0)
    multi = MultiEngine([0, 0])
    pinned = (multi.host_empty(64 << 20), multi.host_empty(32 * 20000))  # portable: both engines' devices
    t0 = last = time.time()
    counts = {"host": 0, "slices": 0, "plan": 0, "large": 0, "chains": 0, "split": 0, "multi": 0, "arena": 0}
    k = 0
    while time.time() - t0 < a.seconds:
        seed = a.seed * 1_000_003 + k
        rng = np.random.default_rng(seed)
        which = ("host", "slices", "plan", "arena", "host", "slices", "plan", "large", "chains", "split", "multi",
                 "arena")[k % 12]
        try:
            if which == "multi":
                case_multi(multi, rng, seed)
            elif which == "arena":
                case_arena(eng, multi, pinned, rng, seed)
            else:
                {"host": case_host, "slices": case_slices, "plan": case_plan, "large": case_large,
                 "chains": case_chains, "split": case_split}[which](eng, rng, seed)
        except AssertionError as e:
            print(e, flush=True)
            sys.exit(1)
        counts[which] += 1
        k += 1
        if time.time() - last > 15:
            print(f"{time.time() - t0:.0f} s: {counts}", flush=True)
            last = time.time()
    multi.close()
    eng.close()
    print(f"soak ok: {k} cases in {time.time() - t0:.0f} s {counts}", flush=True)


if __name__ == "__main__":
    main()
