"""Multi-process (one rank per GPU) request-range sharding with a host gather.

Every rank hashes a contiguous request range on its own GPU (no collective in
the data path: requests are independent, actions.go:22-23).  The digests are
then gathered to ONE rank, the one running the state machine (processResults,
state_machine.go:377-433, consumes them in origin order = rank order).  That
gather is control-plane traffic (32 B per digest) outside the hashing:
torch.distributed.gather -- gloo with CPU tensors, or RCCL ("nccl") with
tensors on the rank's current GPU; no all-gather, no reduction.
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np

from .sharding import shard_ranges

# hash_fn(lo, hi) -> (request digests (hi-lo, 32), batch digests (nb, 32))
HashFn = Callable[[int, int], tuple]


def _gather_rows(rows: np.ndarray, dst: int = 0, group=None) -> Optional[list]:
    """Rows of every rank, in rank order, on rank `dst` (None elsewhere).
    `dst` is a rank of `group` (the group-local rank; the same as the global
    rank with the default group); the collectives take the global rank."""
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    gdst = dst if group is None else dist.get_global_rank(group, dst)
    # RCCL ("nccl") only moves device tensors; gloo moves CPU tensors.
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)] if rank == dst else None
    dist.gather(n, sizes, dst=gdst, group=group)
    # every rank pads to the same row count (gather needs equal shapes): the
    # largest shard, known on dst and sent back as one scalar
    m = torch.tensor([max(int(s.item()) for s in sizes) if rank == dst else 0], dtype=torch.int64, device=dev)
    dist.broadcast(m, src=gdst, group=group)
    buf = torch.zeros((int(m.item()), 32), dtype=torch.uint8, device=dev)
    if rows.shape[0]:
        buf[: rows.shape[0]] = torch.from_numpy(np.ascontiguousarray(rows)).to(dev)
    outs = [torch.zeros_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, outs, dst=gdst, group=group)
    if rank != dst:
        return None
    return [o[: int(s.item())].cpu().numpy() for o, s in zip(outs, sizes)]


def hash_sharded(hash_fn: HashFn, n_req: int, batch_size: int, lengths: Optional[np.ndarray] = None,
                 group=None, dst: int = 0) -> tuple:
    """Run hash_fn on this rank's shard; on rank `dst` (a rank of `group`)
    return (request digests, batch digests) of the whole stream in origin
    order, elsewhere (None, None)."""
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    lo, hi = shard_ranges(n_req, world, batch_size, lengths)[rank]
    req, bat = hash_fn(lo, hi)
    reqs = _gather_rows(np.asarray(req, dtype=np.uint8).reshape(-1, 32), dst, group)
    bats = _gather_rows(np.asarray(bat, dtype=np.uint8).reshape(-1, 32), dst, group)
    if reqs is None:
        return None, None
    return np.concatenate(reqs), np.concatenate(bats)
