#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.json).

Expected digests come from Python ``hashlib`` (OpenSSL 3.0.2 here) — an
implementation independent of both the oracle (oracle/sha256_oracle.c) and the
HIP kernels — over byte layouts restated from the reference:

  kat.json        FIPS 180-2/180-4 example vectors (expected values hard-coded
                  from the standard, cross-checked against hashlib) + boundary
                  lengths 0..130, 183..193, 447..449, 1000, 4095..4097
  layouts.json    testengine request digests (client 0..3, reqNo 0..199;
                  testengine/recorder.go:158-174 payload, state_machine.go:313-317
                  layout), batch digests over them (sequence.go:154-157, incl. null
                  requests client_tracker.go:840-847), an epoch-change payload
                  (stateless.go:311-340), the checkpoint hash chain
                  (testengine/recorder.go:186-256, SHA-256("") after a reset as
                  pinned by testengine/recorder_test.go:83)
  synth.json      synthetic request-stream digests (SURVEY.md §8d generator) for
                  configs 2/3 at chosen indices + seeded log-uniform lengths

Inputs are never stored when they can be regenerated from (seed, index, length).
Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import numpy as np  # noqa: E402

import synth  # noqa: E402
from mirbft_amd import hashdata  # noqa: E402  (pure-python layouts, no native code)


def h(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


NIST = [
    ("", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
    ("abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
    ("abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
    ("abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmnhijklmnoijklmnopjklmnopqklmnopqrlmnopqrsmnopqrstnopqrstu",
     "cf5b16a778af8380036ce59e7b0492370b249b11e8f07a51afac45037afee9d1"),
]
MILLION_A = "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"

BOUNDARY = list(range(0, 131)) + list(range(183, 194)) + [447, 448, 449, 1000, 4095, 4096, 4097]


def make_kat():
    kat = {"nist": [], "million_a": MILLION_A, "boundary": []}
    for msg, want in NIST:
        assert h(msg.encode()) == want, msg
        kat["nist"].append({"ascii": msg, "sha256": want})
    assert h(b"a" * 1_000_000) == MILLION_A
    for n in BOUNDARY:
        kat["boundary"].append({"len": n, "salt": 0, "sha256": h(synth.pattern_bytes(n))})
    return kat


def make_layouts():
    out = {}
    # testengine request digests: BasicRecorder clients 0..3, reqNo 0..199
    reqs = []
    digests = {}
    for c in range(4):
        for r in range(200):
            data = hashdata.request_hash_data(c, r, hashdata.testengine_request_payload(c, r))
            d = hashlib.sha256(hashdata.concat(data)).digest()
            digests[(c, r)] = d
            reqs.append({"client": c, "req_no": r, "sha256": d.hex()})
    out["testengine_requests"] = reqs

    # batches over request digests in (reqNo, client) order; sizes 1, 20, 500,
    # and batches with null requests (empty digests).
    order = [(c, r) for r in range(200) for c in range(4)]
    batches = []

    def add_batch(name, keys):
        ds = [b"" if k is None else digests[k] for k in keys]
        assert any(len(d) for d in ds) or not ds
        batches.append({
            "name": name,
            "entries": [None if k is None else [k[0], k[1]] for k in keys],
            "sha256": h(hashdata.concat(hashdata.batch_hash_data(ds))),
        })

    add_batch("size1", order[:1])
    add_batch("size20", order[:20])
    add_batch("size20_b", order[20:40])
    add_batch("size500", order[100:600])
    add_batch("nulls_mixed", [order[0], None, order[1], None, None, order[2]])
    add_batch("null_first", [None, order[5], order[6]])
    add_batch("size3_odd", order[7:10])
    add_batch("size2_even", order[10:12])
    out["batches"] = batches

    # epoch change payload (stateless.go:311-340)
    cps = [(5 * k, hashlib.sha256(b"cp%d" % k).digest()) for k in range(3)]
    pset = [(1, 10 + k, digests[order[k]]) for k in range(7)]
    qset = [(1, 10 + k, digests[order[k + 7]]) for k in range(5)] + [(0, 3, b"")]
    slices = hashdata.epoch_change_hash_data(4, cps, pset, qset)
    out["epoch_change"] = {
        "new_epoch": 4,
        "checkpoints": [[s, v.hex()] for s, v in cps],
        "p_set": [[e, s, d.hex()] for e, s, d in pset],
        "q_set": [[e, s, d.hex()] for e, s, d in qset],
        "n_slices": len(slices),
        "sha256": h(hashdata.concat(slices)),
    }

    # checkpoint chain: commits of request digests; Sum at each checkpoint,
    # Set() resets the running hash (testengine/recorder.go:186-256).
    commits = [order[i] for i in range(0, 60)]
    chain = []
    running = hashlib.sha256()
    for i, k in enumerate(commits):
        running.update(digests[k])
        if (i + 1) % 20 == 0:
            chain.append({"after_commit": i + 1, "sha256": running.hexdigest()})
            running = hashlib.sha256()
    chain.append({"after_commit": len(commits), "empty_after_reset": running.hexdigest()})
    assert chain[-1]["empty_after_reset"] == NIST[0][1]  # recorder_test.go:83
    out["checkpoint_chain"] = {"commits": [[c, r] for c, r in commits], "checkpoints": chain}
    return out


def make_synth():
    out = {"seed_base": synth.SEED_BASE, "configs": []}
    for cfg, data_len, n_total in ((2, 256, 1 << 20), (3, 4096, 1 << 18)):
        seed = synth.SEED_BASE + cfg
        picks = sorted(set([0, 1, 2, 15, 16, 63, 64, 65, 1000, n_total // 2, n_total - 2, n_total - 1]))
        out["configs"].append({
            "config": cfg,
            "seed": seed,
            "data_len": data_len,
            "n_total": n_total,
            "samples": [{"i": i, "sha256": h(synth.request_message(seed, i, data_len))} for i in picks],
        })
    # first 1024 requests of config 2 -> request digests and BatchSize-20 batch digests
    seed = synth.SEED_BASE + 2
    arena = synth.request_arena(seed, 0, 1024, 256).reshape(1024, 272)
    req = [hashlib.sha256(arena[i].tobytes()).digest() for i in range(1024)]
    bat = [h(b"".join(req[b:b + 20])) for b in range(0, 1024, 20)]
    out["cfg2_prefix"] = {
        "count": 1024,
        "batch_size": 20,
        "request_sha256_of_concat": h(b"".join(req)),
        "batch_sha256": bat,
    }
    # seeded log-uniform lengths 64 B .. 64 KiB (config 5 shape), pattern data
    seed5 = synth.SEED_BASE + 5
    lens = synth.log_uniform_lengths(seed5, 256)
    out["loguniform"] = {
        "seed": seed5,
        "count": 256,
        "lengths": [int(x) for x in lens],
        "sha256": [h(synth.data_bytes(seed5, i, int(n))) for i, n in enumerate(lens)],
    }
    return out


def main():
    for name, fn in (("kat.json", make_kat), ("layouts.json", make_layouts), ("synth.json", make_synth)):
        path = os.path.join(HERE, name)
        with open(path, "w") as f:
            json.dump(fn(), f, indent=1, sort_keys=True)
        print(f"wrote {path} ({os.path.getsize(path)} bytes)")


if __name__ == "__main__":
    main()
