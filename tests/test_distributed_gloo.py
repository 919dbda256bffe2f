"""World-size-2 (and 3) gloo test of the N>1 path: batch-aligned request-range
shards, per-rank hashing, rank-order gather == single-process origin order.

On CPU the per-rank hash function is the oracle (test infrastructure standing in
for each rank's GPU); on a GPU box bench.py runs the same shard arithmetic with
the HIP engine per rank.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle_py
import synth
from mirbft_amd import sharding

SEED = synth.SEED_BASE + 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, n, bs, data_len, q):
    import torch.distributed as dist

    from mirbft_amd.dist import hash_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    stride = 16 + data_len

    def hash_fn(lo, hi):
        arena = oracle_py.gen_requests(SEED, lo, hi - lo, data_len)
        req = oracle_py.hash_requests(arena, np.arange(hi - lo, dtype=np.uint64) * stride, np.full(hi - lo, stride))
        idx, first = sharding.batch_lists(hi - lo, bs)
        return req, oracle_py.batch_digests(req, idx, first)

    req, bat = hash_sharded(hash_fn, n, bs)
    q.put((rank, None if req is None else req.tobytes(), None if bat is None else bat.tobytes()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gather_equals_single_process(world):
    n, bs, data_len = 2003, 20, 256
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, n, bs, data_len, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    stride = 16 + data_len
    arena = oracle_py.gen_requests(SEED, 0, n, data_len)
    want_req = oracle_py.hash_requests(arena, np.arange(n, dtype=np.uint64) * stride, np.full(n, stride))
    idx, first = sharding.batch_lists(n, bs)
    want_bat = oracle_py.batch_digests(want_req, idx, first)
    # gathered to rank 0 only (the state machine's process); no all-gather
    for rank, req, bat in results:
        if rank == 0:
            assert req == want_req.tobytes()
            assert bat == want_bat.tobytes()
        else:
            assert req is None and bat is None, rank


SEED5 = synth.SEED_BASE + 5


def _rank_mixed(rank, world, port, n, q):
    """Config 5's form: one global mixed-length stream, block-balanced shards."""
    import torch.distributed as dist

    from mirbft_amd.dist import hash_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lengths = np.array([oracle_py.mixed_data_len(SEED5, i) + 16 for i in range(n)], dtype=np.uint32)

    def hash_fn(lo, hi):
        arena, off, ln = oracle_py.gen_mixed(SEED5, np.arange(lo, hi, dtype=np.uint64))
        assert np.array_equal(ln, lengths[lo:hi])
        return oracle_py.hash_requests(arena, off, ln), np.zeros((0, 32), np.uint8)

    req, _ = hash_sharded(hash_fn, n, 1, lengths)
    q.put((rank, None if req is None else req.tobytes(), sharding.shard_ranges(n, world, 1, lengths)[rank]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_block_balanced_mixed_stream(world):
    n = 600
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_mixed, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    arena, off, ln = oracle_py.gen_mixed(SEED5, np.arange(n, dtype=np.uint64))
    want = oracle_py.hash_requests(arena, off, ln)
    blk = sharding.blocks_for_len(ln).astype(np.int64)
    shares = []
    for rank, req, (lo, hi) in results:
        assert (req == want.tobytes()) if rank == 0 else req is None, rank
        shares.append(int(blk[lo:hi].sum()))
    # every shard within one request's compressions of the fair share
    assert max(shares) - min(shares) <= 2 * int(blk.max()), shares


def _rank_subgroup(rank, world, port, n, bs, data_len, q):
    """hash_sharded over a subgroup (global ranks 1..world-1) gathering to its
    group rank 1, i.e. global rank 2: dst is a GROUP rank."""
    import torch.distributed as dist

    from mirbft_amd.dist import hash_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    members = list(range(1, world))
    group = dist.new_group(members)
    stride = 16 + data_len

    def hash_fn(lo, hi):
        arena = oracle_py.gen_requests(SEED, lo, hi - lo, data_len)
        req = oracle_py.hash_requests(arena, np.arange(hi - lo, dtype=np.uint64) * stride, np.full(hi - lo, stride))
        idx, first = sharding.batch_lists(hi - lo, bs)
        return req, oracle_py.batch_digests(req, idx, first)

    if rank in members:
        req, bat = hash_sharded(hash_fn, n, bs, group=group, dst=1)
        q.put((rank, None if req is None else req.tobytes(), None if bat is None else bat.tobytes()))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_gather_subgroup_dst_is_group_rank():
    world, n, bs, data_len = 3, 1001, 20, 64
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_subgroup, args=(r, world, port, n, bs, data_len, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world - 1)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    stride = 16 + data_len
    arena = oracle_py.gen_requests(SEED, 0, n, data_len)
    want_req = oracle_py.hash_requests(arena, np.arange(n, dtype=np.uint64) * stride, np.full(n, stride))
    idx, first = sharding.batch_lists(n, bs)
    want_bat = oracle_py.batch_digests(want_req, idx, first)
    for rank, req, bat in results:
        if rank == 2:  # group rank 1
            assert req == want_req.tobytes() and bat == want_bat.tobytes()
        else:
            assert req is None and bat is None, rank
