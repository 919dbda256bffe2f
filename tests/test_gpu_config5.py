"""BASELINE config 5 at one rank's full workload: the 10^8-request mixed-size
stream (64 B - 64 KB data, log-uniform) cut for 8 GPUs by the block-balanced
sharder, and rank 3's shard (~12.5 M requests, ~123 GB) generated into HBM
and hashed in the product launch (64-bit addressed LDS loader, one launch,
longest-first bucket order), as bench.py --config 5 does per rank.  1,024
sampled digests plus the shard's first and last are compared with the
oracle (processor.go:133-143 over the same bytes).

Run on an MI355X:  python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
"""
import numpy as np
import pytest

import oracle_py
from mirbft_amd import bucket_order, sharding

pytestmark = pytest.mark.gpu

SEED5 = 0x6D69726266740005
N_GLOBAL, WORLD, RANK = 10**8, 8, 3


def test_config5_rank_shard_full_size(engine):
    import torch

    dev = torch.device("cuda", torch.cuda.current_device())
    # the global stream's lengths, on the device (the generator bench.py uses)
    d_all = torch.empty(N_GLOBAL, dtype=torch.int32, device=dev)
    engine.synth_mixed_lengths_device(SEED5, 0, N_GLOBAL, d_all.data_ptr())
    engine.sync()
    lens_all = d_all.cpu().numpy().view(np.uint32)
    del d_all
    probe = np.array([0, 1, 12_345_678, N_GLOBAL - 1], dtype=np.int64)
    assert [int(lens_all[i]) for i in probe] == [16 + oracle_py.mixed_data_len(SEED5, int(i)) for i in probe]
    lo, hi = sharding.shard_ranges(N_GLOBAL, WORLD, 1, lens_all)[RANK]
    n = hi - lo
    assert abs(n - N_GLOBAL // WORLD) < 0.01 * N_GLOBAL // WORLD
    ln = np.ascontiguousarray(lens_all[lo:hi])
    del lens_all
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(ln[:-1], out=off[1:])
    total = int(off[-1]) + int(ln[-1])
    assert total > 100e9  # ~123 GB device-resident
    d_len = torch.from_numpy(ln.view(np.int32)).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_arena = torch.empty(total, dtype=torch.uint8, device=dev)
    engine.synth_mixed_device(SEED5, lo, n, d_off.data_ptr(), d_arena.data_ptr())
    order, _ = bucket_order(ln)
    d_order = torch.from_numpy(order.view(np.int32)).to(dev)
    d_out = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    engine.sync()
    torch.cuda.synchronize()
    engine.hash_batch_device(d_arena.data_ptr(), total, d_off.data_ptr(), d_len.data_ptr(), d_order.data_ptr(), n,
                             d_out.data_ptr())
    engine.sync()
    rng = np.random.default_rng(5)
    pick = np.unique(np.concatenate([rng.choice(n, 1024, replace=False), [0, 1, n - 1]]))
    got = d_out[torch.from_numpy(pick).to(dev)].cpu().numpy()
    arena, o_off, o_ln = oracle_py.gen_mixed(SEED5, (lo + pick).astype(np.uint64))
    assert np.array_equal(o_ln, ln[pick])
    want = oracle_py.hash_requests(arena, o_off, o_ln, threads=8)
    assert np.array_equal(got, want)
    # and every digest was written (none left at the zero fill)
    assert not bool((d_out == 0).all(dim=1).any())
