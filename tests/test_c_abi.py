"""The cgo call sequence of INTEGRATION.md's Go binding, made from C: gcc
compiles tests/c/cgo_sequence.c against include/mirsha.h and links
libmirsha.so (CPU test); on the GPU the program runs with no Python in the
process and its digests are compared with the golden testengine request
digests (tests/golden/layouts.json, hashlib-made from the reference's layouts,
testengine/recorder.go:158-174 and state_machine.go:313-317)."""
import json
import os
import subprocess

import numpy as np
import pytest

import oracle_py
from chunking import plan_chunks
from mirbft_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c", "cgo_sequence.c")
PATH_SRC = os.path.join(ROOT, "tests", "c", "cgo_path.c")


def build(out_dir, src=SRC, name="cgo_sequence") -> str:
    exe = os.path.join(str(out_dir), name)
    subprocess.run(["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror", "-pthread", "-I",
                    os.path.join(ROOT, "include"), src, "-L", _lib.LIB_DIR, "-lmirsha", "-Wl,-rpath," + _lib.LIB_DIR,
                    "-o", exe], check=True)
    return exe


def test_cgo_sequence_compiles_and_links(tmp_path):
    exe = build(tmp_path)
    # every mirsha_* symbol the program calls resolves in libmirsha.so
    ldd = subprocess.run(["ldd", exe], capture_output=True, text=True, check=True).stdout
    assert "libmirsha.so" in ldd and "not found" not in ldd


@pytest.mark.gpu
def test_cgo_sequence_on_gpu(tmp_path, layouts):
    exe = build(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert "fips ok" in lines and lines[-1] == "sequence ok"
    want = {200 * e["client"] + e["req_no"]: e["sha256"] for e in layouts["testengine_requests"]}
    assert len(want) == 800
    for tag in ("req", "chunk", "async", "multi", "cmulti", "amulti"):
        got = {int(i): h for t, i, h in (ln.split() for ln in lines if ln.startswith(tag + " "))}
        assert got == want, tag


def test_cgo_path_compiles_and_links(tmp_path):
    exe = build(tmp_path, PATH_SRC, "cgo_path")
    ldd = subprocess.run(["ldd", exe], capture_output=True, text=True, check=True).stdout
    assert "libmirsha.so" in ldd and "not found" not in ldd


@pytest.mark.gpu
@pytest.mark.parametrize("stores", ["plain", "nt"])
def test_cgo_path_on_gpu(tmp_path, stores):
    """The binding's HashBatch from C: the chunked form INTEGRATION.md now
    gives (packing of chunk k+1 overlapping chunk k's mirsha_submit_batch),
    round 4's one-call form, the serial form, the library-packed
    mirsha_hash_slices and the multi-device twin (mirsha_submit_arena_multi,
    device 0 twice): every leg agrees with the serial one (checked in the
    program) and the digests are the oracle's.  A 1 MiB chunk budget gives 28
    chunks, far more than the 4-slot ring.  stores "nt": the workers stream
    the arena with non-temporal stores through a per-worker window."""
    exe = build(tmp_path, PATH_SRC, "cgo_path")
    n, data_len = 100_003, 256
    r = subprocess.run([exe, str(n), str(data_len), "8", "2", "1", stores], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.splitlines()[-1])
    assert line["requests"] == n and line["parallel"]["ms"] > 0 and line["pack_stores"] == stores
    # chunks end at block boundaries (blocks of ceil(n / 4096) requests); the
    # first two have a quarter and a half of the budget
    chunks = plan_chunks(np.full(n, 16 + data_len), 1 << 20)
    assert line["parallel"]["chunks"] == len(chunks) == line["multi"]["chunks"] > 20
    assert all(hi > lo for lo, hi, _ in chunks)
    arena = oracle_py.gen_requests(0x6D69726266740002, 0, 4, data_len)
    stride = 16 + data_len
    want = oracle_py.hash_requests(arena, np.arange(4, dtype=np.uint64) * stride, np.full(4, stride))
    assert line["sample"].split(",") == [w.tobytes().hex() for w in want]


def test_plan_chunks_splits_only_oversized_blocks():
    n, big_every = 20_000, 1000
    lens = np.full(n, 272)
    lens[big_every - 1::big_every] = 16 + 3 * (1 << 20)
    chunks = plan_chunks(lens, 1 << 20)
    # contiguous, covering every request once
    assert chunks[0][0] == 0 and chunks[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(chunks, chunks[1:]))
    # every chunk fits a budget unless it is one request; parts exist only for the 20 big blocks
    for lo, hi, whole in chunks:
        if not whole and hi - lo > 1:
            assert lens[lo:hi].sum() <= 1 << 20
    parts = [c for c in chunks if not c[2]]
    assert sum(1 for lo, hi, _ in parts if hi - lo == 1 and lens[lo] > 1 << 20) == n // big_every
    # the uniform config-2 shape never splits
    assert all(w for _, _, w in plan_chunks(np.full(1 << 20, 272), 32 << 20))


@pytest.mark.gpu
def test_cgo_path_large_messages_split_blocks(tmp_path):
    """a block holding more than a chunk budget (large messages) is
    cut at request boundaries, so no mirsha_submit_batch outgrows one device
    arena; every leg still agrees, and the large request's digest is the
    oracle's."""
    exe = build(tmp_path, PATH_SRC, "cgo_path")
    n, data_len, big_every, big_len = 20_000, 256, 1000, 3 * (1 << 20)
    r = subprocess.run([exe, str(n), str(data_len), "8", "1", "1", "nt", str(big_every), str(big_len)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.splitlines()[-1])
    lens = np.full(n, 16 + data_len)
    lens[big_every - 1::big_every] = 16 + big_len
    chunks = plan_chunks(lens, 1 << 20)
    assert line["parallel"]["chunks"] == len(chunks) == line["multi"]["chunks"]
    assert any(not w for _, _, w in chunks)
    sb = line["sample_big"]
    assert sb["index"] == big_every - 1
    big = oracle_py.gen_requests(0x6D69726266740002, big_every - 1, 1, big_len)
    want = oracle_py.hash_requests(big, np.zeros(1, np.uint64), np.full(1, 16 + big_len))
    assert sb["sha256"] == want[0].tobytes().hex()
