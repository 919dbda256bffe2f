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
    br = -(-n // 4096)
    nb = -(-n // br)
    bsum = [min(br, n - b * br) * (16 + data_len) for b in range(nb)]
    want_chunks, b0 = 0, 0
    while b0 < nb:
        budget = (1 << 20) >> (2 - want_chunks) if want_chunks < 2 else 1 << 20
        acc, b1 = bsum[b0], b0 + 1
        while b1 < nb and acc < budget:
            acc += bsum[b1]
            b1 += 1
        want_chunks, b0 = want_chunks + 1, b1
    assert line["parallel"]["chunks"] == want_chunks == line["multi"]["chunks"] > 20
    arena = oracle_py.gen_requests(0x6D69726266740002, 0, 4, data_len)
    stride = 16 + data_len
    want = oracle_py.hash_requests(arena, np.arange(4, dtype=np.uint64) * stride, np.full(4, stride))
    assert line["sample"].split(",") == [w.tobytes().hex() for w in want]
