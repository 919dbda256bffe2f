"""Multi-process (one rank per GPU) request-range sharding with a host gather.

Every rank hashes a contiguous, batch-aligned request range on its own GPU
(no collective in the data path: requests are independent, actions.go:22-23);
digests are gathered to every rank in rank order, which is origin order.
The gather is control-plane traffic (32 B per digest) over torch.distributed —
gloo with CPU tensors, or RCCL ("nccl") with tensors on the rank's current GPU.
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np

from .sharding import shard_ranges

# hash_fn(lo, hi) -> (request digests (hi-lo, 32), batch digests (nb, 32))
HashFn = Callable[[int, int], tuple]


def _all_gather_rows(rows: np.ndarray, group=None) -> list:
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    # RCCL ("nccl") only moves device tensors; gloo moves CPU tensors.
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    m = max(int(s.item()) for s in sizes)
    buf = torch.zeros((m, 32), dtype=torch.uint8, device=dev)
    if rows.shape[0]:
        buf[: rows.shape[0]] = torch.from_numpy(np.ascontiguousarray(rows)).to(dev)
    outs = [torch.zeros((m, 32), dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    return [o[: int(s.item())].cpu().numpy() for o, s in zip(outs, sizes)]


def hash_sharded(hash_fn: HashFn, n_req: int, batch_size: int, lengths: Optional[np.ndarray] = None,
                 group=None) -> tuple:
    """Run hash_fn on this rank's shard, gather (requests, batches) in origin order."""
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    lo, hi = shard_ranges(n_req, world, batch_size, lengths)[rank]
    req, bat = hash_fn(lo, hi)
    reqs = _all_gather_rows(np.asarray(req, dtype=np.uint8).reshape(-1, 32), group)
    bats = _all_gather_rows(np.asarray(bat, dtype=np.uint8).reshape(-1, 32), group)
    return np.concatenate(reqs), np.concatenate(bats)
