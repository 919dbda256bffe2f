"""CPU tests of bench.py's control-plane pieces (verdict r5 items 3 and 5):
the per-rank self-check windows, the device-identity check, the launcher's
device count in a child process, and the OpenSSL EVP baseline loop
(oracle/evp_loop.c) against the oracle."""
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402
import oracle_py as o  # noqa: E402
from mirbft_amd import sharding  # noqa: E402


@pytest.mark.parametrize("n,bs", [(1000, 20), (1010, 20), (1 << 20, 20), (1 << 18, 500), (7, 20), (20, 20)])
def test_check_windows_cover_both_ends(n, bs):
    nb = (n + bs - 1) // bs
    w = bench.check_windows(nb, bs, seed=3)
    assert w[0][0] == 0
    assert w[-1][1] == nb  # the final (possibly partial) batch is always checked
    assert all(0 <= b0 < b1 <= nb for b0, b1 in w)
    assert 2 <= len(w) <= 6 or nb <= max(1, 256 // bs)


def _rank_digests(seed, first_req, n, data_len, bs):
    idx, first = sharding.batch_lists(n, bs)
    stride = 16 + data_len
    req = o.hash_requests(o.gen_requests(seed, first_req, n, data_len), np.arange(n, dtype=np.uint64) * stride,
                          np.full(n, stride))
    return idx, first, req, o.batch_digests(req, idx, first)


@pytest.mark.parametrize("n", [1000, 1010, 333])
def test_check_batch_windows_accepts_oracle_and_catches_the_partial_batch(n):
    seed, first_req, data_len, bs = bench.SEED_BASE + 2, 5 * n, 256, 20
    idx, first, req, bat = _rank_digests(seed, first_req, n, data_len, bs)
    assert bench.check_batch_windows(seed, first_req, data_len, idx, first, req, bat)
    bad = bat.copy()
    bad[-1, 31] ^= 0x80  # the final batch (partial when 20 does not divide n)
    assert not bench.check_batch_windows(seed, first_req, data_len, idx, first, req, bad)
    badr = req.copy()
    badr[n - 1, 0] ^= 1  # the range's last request
    assert not bench.check_batch_windows(seed, first_req, data_len, idx, first, badr, bat)
    badf = req.copy()
    badf[0, 0] ^= 1  # its first request
    assert not bench.check_batch_windows(seed, first_req, data_len, idx, first, badf, bat)
    # another rank's range (wrong first request) must not pass
    assert not bench.check_batch_windows(seed, first_req + 1, data_len, idx, first, req, bat)


def test_device_identity_check():
    pr = [{"device_uuid": "GPU-aa"}, {"device_uuid": "GPU-bb"}]
    assert bench.device_identity_check(pr, False)["distinct"] is True
    pr2 = [{"device_uuid": "GPU-aa"}, {"device_uuid": "GPU-aa"}]
    assert bench.device_identity_check(pr2, False)["distinct"] is False
    assert bench.device_identity_check(pr2, True)["distinct"] is None  # rehearsal: one device on purpose
    # zero UUIDs fall back to the PCI bus id
    pr3 = [{"device_uuid": "00000000-0000-0000", "pci_bus_id": 3}, {"device_uuid": "", "pci_bus_id": 4}]
    assert bench.device_identity_check(pr3, False)["distinct"] is True
    pr4 = [{"device_uuid": "", "pci_bus_id": None}, {"device_uuid": "", "pci_bus_id": None}]
    assert bench.device_identity_check(pr4, False)["distinct"] is None
    assert bench.device_identity_check(pr[:1], False)["distinct"] is True


def test_launcher_counts_devices_without_torch_in_the_parent():
    """verdict r5 item 3(c): the launching process must never initialise HIP;
    it does not even import torch (the count runs in a child)."""
    code = ("import sys; sys.path.insert(0, %r); sys.argv = ['bench.py', '--gpus', '2', '--steps', '1']; "
            "import bench; a = bench.parse(); rc = bench.launch_ranks(a); "
            "print('torch' in sys.modules, rc)") % ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "MIRSHA_BENCH_DEVICE",
                                                             "MIRSHA_BENCH_COUNT_STUB")}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split()[-2:] == ["False", "2"], r.stdout  # no GPU here: 0 visible < 2 -> refused
    assert "0 device(s) visible" in r.stderr


def test_count_devices_child_process():
    assert bench.count_devices() == 0  # no GPU in this container; the child's torch says 0


def test_evp_loop_matches_oracle_and_hashlib():
    rng = np.random.default_rng(11)
    lens = np.r_[np.arange(0, 200), rng.integers(0, 5000, 60)].astype(np.uint32)
    off = np.zeros(lens.size, np.uint64)
    np.cumsum(lens[:-1], out=off[1:])
    arena = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    want = o.hash_requests(arena, off, lens)
    for threads in (1, 4):
        for split in (True, False):
            assert np.array_equal(o.evp_hash_requests(arena, off, lens, threads=threads, split=split), want)
    assert bytes(o.evp_hash_requests(arena, off[:1], np.zeros(1, np.uint32))[0]) == hashlib.sha256(b"").digest()
    # batch digests with null requests (client_tracker.go:840-847)
    idx = np.array([0, 1, o.NULL, 2, o.NULL, o.NULL, 3], np.uint32)
    first = np.array([0, 3, 4, 6, 7], np.uint32)
    assert np.array_equal(o.evp_batch_digests(want, idx, first), o.batch_digests(want, idx, first))
    assert o.evp_version().startswith("OpenSSL")


def test_evp_pool_on_config2_sample():
    n, data_len = 4096, 256
    stride = 16 + data_len
    arena = o.gen_requests(bench.SEED_BASE + 2, 0, n, data_len)
    off = np.arange(n, dtype=np.uint64) * stride
    ln = np.full(n, stride, np.uint32)
    assert np.array_equal(o.evp_hash_requests(arena, off, ln, threads=8), o.hash_requests(arena, off, ln))


@pytest.mark.parametrize("steps,every,want", [(20, 4, [3, 7, 11, 15, 19]), (20, 1, list(range(20))),
                                              (5, 4, [3]), (3, 4, [2]), (1, 4, [0]), (50, 4, list(range(3, 50, 4)))])
def test_event_steps_sample_every_kth_never_the_first(steps, every, want):
    got = bench.event_steps(steps, every)
    assert got == want
    assert got and (0 not in got or steps == 1 or every == 1)
