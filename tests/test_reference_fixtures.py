"""Layouts pinned by the reference's own tests (tests/golden/reference_fixtures.json).

sequence_test.go:39-88 asserts the exact HashRequest that sequence.allocate
emits for a batch of two RequestAcks: Data is one slice per ack digest, in
order (sequence.go:154-157).  The reference asserts no digest value there, so
the digest is checked against hashlib's SHA-256 of the concatenated slices
(what processor.go:133-143 computes); on the GPU the same HashRequest goes
through the Processor mirror and must come back with its Request
back-pointer."""
import hashlib

import pytest

import oracle_py
from mirbft_amd import hashdata


def _fixture(golden_dir):
    import json
    import os

    with open(os.path.join(golden_dir, "reference_fixtures.json")) as f:
        return json.load(f)["sequence_allocate"]


@pytest.fixture(scope="module")
def seq_alloc():
    import os

    return _fixture(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))


def test_batch_layout_matches_sequence_test(seq_alloc):
    acks = [a["digest_ascii"].encode() for a in seq_alloc["request_acks"]]
    data = hashdata.batch_hash_data(acks)
    assert data == [d.encode() for d in seq_alloc["expected_hash_request"]["data_ascii"]]


def test_batch_digest_of_the_fixture_on_the_oracle(seq_alloc):
    data = [d.encode() for d in seq_alloc["expected_hash_request"]["data_ascii"]]
    want = hashlib.sha256(b"".join(data)).digest()
    assert oracle_py.hash_messages([b"".join(data)])[0].tobytes() == want


@pytest.mark.gpu
def test_batch_fixture_through_the_processor(engine, seq_alloc):
    from mirbft_amd import Actions, HashRequest, Processor

    data = [d.encode() for d in seq_alloc["expected_hash_request"]["data_ascii"]]
    req = HashRequest(data=data, origin=seq_alloc["expected_hash_request"]["origin"])
    res = Processor(engine).process(Actions(hash=[req]))
    assert len(res.digests) == 1
    assert res.digests[0].request is req
    assert bytes(res.digests[0].digest) == hashlib.sha256(b"".join(data)).digest()
