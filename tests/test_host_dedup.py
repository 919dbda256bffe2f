"""Content-addressed dedup plan (mirsha_dedup_plan, host code only -- no GPU):
the grouping behind mirsha_hash_slices_dedup / MIRSHA_SUBMIT_DEDUP.  Equal
request BYTES (however sliced) share one representative, the smallest index;
different bytes never do, fingerprint collisions included."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from mirbft_amd import SliceArrays, dedup_plan, hashdata
from mirbft_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def python_plan(requests):
    seen, rep = {}, []
    for i, r in enumerate(requests):
        b = b"".join(bytes(s) for s in r)
        rep.append(seen.setdefault(b, i))
    return np.array(rep, dtype=np.uint32), len(seen)


def random_requests(seed, n=300, contents=12):
    rng = np.random.default_rng(seed)
    pool = [rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes() for _ in range(contents)]
    # near-duplicates: same length, one byte different; and prefixes
    pool.append(pool[0][:-1] + bytes([pool[0][-1] ^ 1]) if pool[0] else b"\x01")
    pool.append(pool[1][: len(pool[1]) // 2])
    reqs = []
    for _ in range(n):
        b = pool[int(rng.integers(0, len(pool)))]
        cuts = sorted(int(x) for x in rng.integers(0, len(b) + 1, int(rng.integers(0, 5))))
        parts, last = [], 0
        for c in cuts + [len(b)]:
            parts.append(b[last:c])
            last = c
        if rng.random() < 0.2:
            parts.insert(int(rng.integers(0, len(parts) + 1)), b"")
        reqs.append(parts)
    return reqs


def test_slicing_does_not_matter():
    reqs = [[b"ab", b"c"], [b"abc"], [b""], [b"a", b"bc"], [], [b"xyz"], [b"abd"], [b"", b"abc", b""]]
    rep, u = dedup_plan(reqs)
    assert rep.tolist() == [0, 0, 2, 0, 2, 5, 6, 0]
    assert u == 4


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_random_against_python(seed):
    reqs = random_requests(seed)
    rep, u = dedup_plan(reqs)
    want, wu = python_plan(reqs)
    assert rep.tolist() == want.tolist() and u == wu


def test_word_alignment_across_slices():
    """Same 40 bytes cut at every position into 2 and 3 slices: one class."""
    b = bytes(range(40))
    reqs = [[b]] + [[b[:i], b[i:]] for i in range(41)] + [[b[:i], b[i:j], b[j:]] for i in range(0, 41, 3)
                                                          for j in range(i, 41, 5)]
    rep, u = dedup_plan(reqs)
    assert u == 1 and set(rep.tolist()) == {0}


def test_weak_fingerprint_collisions_resolved_exactly():
    """MIRSHA_DEDUP_WEAK_FP=1 makes every fingerprint equal, so every
    same-length pair is a collision that only the byte comparison separates."""
    code = (
        "import sys; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
        "import test_host_dedup as t\n"
        "from mirbft_amd import dedup_plan\n"
        "for seed in (0, 1, 2):\n"
        "    reqs = t.random_requests(seed, n=200)\n"
        "    rep, u = dedup_plan(reqs)\n"
        "    want, wu = t.python_plan(reqs)\n"
        "    assert rep.tolist() == want.tolist() and u == wu, seed\n"
        "print('ok')\n" % (ROOT, os.path.join(ROOT, "tests"))
    )
    env = dict(os.environ, MIRSHA_AB="1", MIRSHA_DEDUP_WEAK_FP="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr


@pytest.mark.parametrize("weak", ["0", "1"])
def test_streamed_segments(weak):
    """The scan in segments of a few slices (test hook MIRSHA_DEDUP_SEGMENT_SLICES,
    read once per process, hence a subprocess): heads of later segments,
    matches confirmed inside the scan against heads of earlier segments, and
    (weak fingerprints) collisions across segments all give the plan of the
    one-segment scan; a malformed request in a later segment is still found."""
    code = (
        "import sys, ctypes; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
        "import numpy as np\n"
        "import test_host_dedup as t\n"
        "from mirbft_amd import dedup_plan, SliceArrays, _lib\n"
        "for seed in (0, 1, 2, 3):\n"
        "    reqs = t.random_requests(seed, n=200)\n"
        "    rep, u = dedup_plan(reqs)\n"
        "    want, wu = t.python_plan(reqs)\n"
        "    assert rep.tolist() == want.tolist() and u == wu, seed\n"
        "sl = SliceArrays.from_requests([[b'ab', b'c']] * 30)\n"
        "ptr = sl.ptr.copy(); ptr[47] = 0\n"
        "rep = np.zeros(30, dtype=np.uint32); u = ctypes.c_uint32(0)\n"
        "rc = _lib.load().mirsha_dedup_plan(ptr.ctypes.data, sl.len.ctypes.data, sl.first.ctypes.data, 30,\n"
        "                                   rep.ctypes.data, ctypes.byref(u))\n"
        "assert rc == _lib.MIRSHA_EINVAL, rc\n"
        "print('ok')\n" % (ROOT, os.path.join(ROOT, "tests"))
    )
    env = dict(os.environ, MIRSHA_AB="1", MIRSHA_DEDUP_SEGMENT_SLICES="5", MIRSHA_DEDUP_WEAK_FP=weak)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr


def test_epoch_change_cycle_parallel_pass():
    """Config-4 shape (acks of every origin relayed by every source), large
    enough (> 4 MiB) for the multi-threaded fingerprint / confirm passes."""
    n_nodes, n_req = 8, 96
    buf, so, sl, first, origin = hashdata.epoch_change_cycle(n_nodes, n_req, 3, 700, 700)
    assert buf.size > (4 << 20)
    arrays = SliceArrays.from_buffer(buf, so, sl, first)
    rep, u = dedup_plan(arrays)
    assert u == n_nodes
    assert rep.tolist() == [int(o) for o in origin]  # origin o first appears at index o
    # flip one byte of request 50's copy: it becomes distinct
    buf2 = buf.copy()
    r = 50
    buf2[int(so[first[r] + 5]) + 3] ^= 0xFF
    rep2, u2 = dedup_plan(SliceArrays.from_buffer(buf2, so, sl, first))
    assert u2 == n_nodes + 1 and rep2[r] == r
    assert all(rep2[i] == rep[i] for i in range(n_req) if i != r)


def test_empty_and_invalid():
    rep, u = dedup_plan([])
    assert rep.size == 0 and u == 0
    lib = _lib.load()
    rep = np.zeros(2, dtype=np.uint32)
    u = ctypes.c_uint32(0)
    bad_first = np.array([1, 1, 1], dtype=np.uint32)  # first[0] must be 0
    assert lib.mirsha_dedup_plan(None, None, bad_first.ctypes.data, 2, rep.ctypes.data, ctypes.byref(u)) == \
        _lib.MIRSHA_EINVAL
    non_mono = np.array([0, 2, 1], dtype=np.uint32)
    lens = np.zeros(2, dtype=np.uint64)
    ptrs = np.zeros(2, dtype=np.uint64)
    assert lib.mirsha_dedup_plan(ptrs.ctypes.data, lens.ctypes.data, non_mono.ctypes.data, 2, rep.ctypes.data,
                                 ctypes.byref(u)) == _lib.MIRSHA_EINVAL


def test_host_mirror_exports_async_and_dedup_entry():
    host = ctypes.CDLL(_lib.HOST_LIB_PATH)
    assert hasattr(host, "mirbft_host_process_ex")
