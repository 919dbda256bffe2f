"""Pin the CPU oracle against the committed golden fixtures (CPU only).

The oracle restates processor.go:129-143 + FIPS 180-4; the fixtures come from
hashlib (tests/golden/make_golden.py) and the FIPS example vectors.
"""
import hashlib

import numpy as np
import pytest

import oracle_py
import synth
from mirbft_amd import hashdata

IMPLS = [0, 1]


@pytest.fixture(params=IMPLS, ids=["scalar", "shani"])
def impl(request):
    if request.param == 1 and not oracle_py.has_shani():
        pytest.skip("CPU has no SHA extensions")
    oracle_py.force_impl(request.param)
    yield request.param
    oracle_py.force_impl(-1)


def test_nist_vectors(kat, impl):
    msgs = [v["ascii"].encode() for v in kat["nist"]]
    got = oracle_py.hash_messages(msgs)
    for v, d in zip(kat["nist"], got):
        assert d.tobytes().hex() == v["sha256"]


def test_million_a(kat, impl):
    got = oracle_py.hash_messages([b"a" * 1_000_000])
    assert got[0].tobytes().hex() == kat["million_a"]


def test_empty_is_reference_checkpoint_value(impl):
    # testengine/recorder_test.go:83 — the only digest value the reference pins.
    got = oracle_py.hash_messages([b""])
    assert got[0].tobytes().hex() == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"


def test_boundary_lengths(kat, impl):
    vs = kat["boundary"]
    got = oracle_py.hash_messages([synth.pattern_bytes(v["len"], v["salt"]) for v in vs])
    for v, d in zip(vs, got):
        assert d.tobytes().hex() == v["sha256"], v["len"]


def test_testengine_request_digests(layouts, impl):
    rs = layouts["testengine_requests"]
    msgs = [hashdata.concat(hashdata.request_hash_data(r["client"], r["req_no"],
                                                       hashdata.testengine_request_payload(r["client"], r["req_no"])))
            for r in rs]
    assert all(len(m) == 33 for m in msgs)  # 16 + 17 bytes, one block
    got = oracle_py.hash_messages(msgs)
    for r, d in zip(rs, got):
        assert d.tobytes().hex() == r["sha256"]


def _req_digest_table(layouts):
    keys = {(r["client"], r["req_no"]): i for i, r in enumerate(layouts["testengine_requests"])}
    table = np.array([bytes.fromhex(r["sha256"]) for r in layouts["testengine_requests"]], dtype=object)
    dig = np.frombuffer(b"".join(table), dtype=np.uint8).reshape(-1, 32)
    return keys, dig


def test_batch_digests_with_nulls(layouts, impl):
    keys, dig = _req_digest_table(layouts)
    idx, first = [], [0]
    for b in layouts["batches"]:
        for e in b["entries"]:
            idx.append(oracle_py.NULL if e is None else keys[(e[0], e[1])])
        first.append(len(idx))
    got = oracle_py.batch_digests(dig, idx, first)
    for b, d in zip(layouts["batches"], got):
        assert d.tobytes().hex() == b["sha256"], b["name"]


def test_epoch_change_payload(layouts, impl):
    ec = layouts["epoch_change"]
    slices = hashdata.epoch_change_hash_data(
        ec["new_epoch"],
        [(s, bytes.fromhex(v)) for s, v in ec["checkpoints"]],
        [(e, s, bytes.fromhex(d)) for e, s, d in ec["p_set"]],
        [(e, s, bytes.fromhex(d)) for e, s, d in ec["q_set"]],
    )
    assert len(slices) == ec["n_slices"]
    got = oracle_py.hash_messages([hashdata.concat(slices)])
    assert got[0].tobytes().hex() == ec["sha256"]


def test_checkpoint_chain(layouts, impl):
    keys, dig = _req_digest_table(layouts)
    cc = layouts["checkpoint_chain"]
    commits = [keys[(c, r)] for c, r in cc["commits"]]
    idx, first, want = [], [0], []
    start = 0
    for cp in cc["checkpoints"]:
        end = cp["after_commit"]
        idx += commits[start:end]
        first.append(len(idx))
        want.append(cp.get("sha256") or cp.get("empty_after_reset"))
        start = end
    got = oracle_py.batch_digests(dig, idx, first)
    assert [d.tobytes().hex() for d in got] == want


def test_generator_matches_synth(synth_fx):
    for cfg in synth_fx["configs"]:
        for s in cfg["samples"][:6]:
            arena = oracle_py.gen_requests(cfg["seed"], s["i"], 1, cfg["data_len"])
            assert arena.tobytes() == synth.request_message(cfg["seed"], s["i"], cfg["data_len"])
            assert hashlib.sha256(arena.tobytes()).hexdigest() == s["sha256"]


def test_cfg2_prefix(synth_fx, impl):
    fx = synth_fx["cfg2_prefix"]
    n = fx["count"]
    arena = oracle_py.gen_requests(synth.SEED_BASE + 2, 0, n, 256)
    off = np.arange(n, dtype=np.uint64) * 272
    req = oracle_py.hash_requests(arena, off, np.full(n, 272))
    assert hashlib.sha256(req.tobytes()).hexdigest() == fx["request_sha256_of_concat"]
    first = list(range(0, n, fx["batch_size"])) + [n]
    bat = oracle_py.batch_digests(req, np.arange(n), first)
    assert [d.tobytes().hex() for d in bat] == fx["batch_sha256"]


def test_loguniform(synth_fx, impl):
    fx = synth_fx["loguniform"]
    lens = synth.log_uniform_lengths(fx["seed"], fx["count"])
    assert [int(x) for x in lens] == fx["lengths"]
    msgs = [synth.data_bytes(fx["seed"], i, int(n)) for i, n in enumerate(lens)]
    got = oracle_py.hash_messages(msgs)
    assert [d.tobytes().hex() for d in got] == fx["sha256"]


def test_multithreaded_preserves_origin_order(impl):
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 3000, 500).astype(np.uint32)
    off = np.zeros(500, dtype=np.uint64)
    np.cumsum(lens[:-1], out=off[1:])
    arena = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    a = oracle_py.hash_requests(arena, off, lens)
    b = oracle_py.hash_requests(arena, off, lens, threads=4)
    assert np.array_equal(a, b)
    for i in (0, 17, 499):
        assert a[i].tobytes() == hashlib.sha256(arena[off[i]:off[i] + lens[i]].tobytes()).digest()
