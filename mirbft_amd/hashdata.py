"""Byte layouts of the reference's hash producers (what `HashRequest.Data` holds).

These are the callers on the producer side of the hot path; each function
returns the ``[][]byte`` slice list exactly as the reference builds it, so that
hashing ``concat(slices)`` reproduces the reference's digest.
"""
from __future__ import annotations

import struct
from typing import Iterable, Sequence


def uint64_to_bytes(value: int) -> bytes:
    """proposer.go:16-20 — binary.LittleEndian.PutUint64 into 8 bytes."""
    return struct.pack("<Q", value & 0xFFFFFFFFFFFFFFFF)


def request_hash_data(client_id: int, req_no: int, data: bytes) -> list[bytes]:
    """StateMachine.propose, state_machine.go:313-317 (and the identical VerifyRequest
    layout of clientTracker.applyForwardRequest, client_tracker.go:618-622)."""
    return [uint64_to_bytes(client_id), uint64_to_bytes(req_no), bytes(data)]


def testengine_request_payload(client_id: int, req_no: int) -> bytes:
    """RecorderClient.RequestByReqNo payload, testengine/recorder.go:164-167:
    LE64(client) || "-" || LE64(reqNo) (17 bytes)."""
    return uint64_to_bytes(client_id) + b"-" + uint64_to_bytes(req_no)


def batch_hash_data(ack_digests: Sequence[bytes]) -> list[bytes]:
    """sequence.allocate, sequence.go:154-157 (and batch_tracker.go:147-150): one
    slice per RequestAck digest; a null request's digest is empty
    (client_tracker.go:840-847).  Callers must not hash an empty batch
    (sequence.go:148-152 skips it)."""
    return [bytes(d) for d in ack_digests]


def epoch_change_hash_data(
    new_epoch: int,
    checkpoints: Iterable[tuple[int, bytes]],
    p_set: Iterable[tuple[int, int, bytes]],
    q_set: Iterable[tuple[int, int, bytes]],
) -> list[bytes]:
    """epochChangeHashData, stateless.go:311-340:
    [LE64(NewEpoch), {LE64(cp.SeqNo), cp.Value}..., {LE64(Epoch), LE64(SeqNo), Digest} for PSet, then QSet]."""
    out = [uint64_to_bytes(new_epoch)]
    for seq_no, value in checkpoints:
        out += [uint64_to_bytes(seq_no), bytes(value)]
    for epoch, seq_no, digest in p_set:
        out += [uint64_to_bytes(epoch), uint64_to_bytes(seq_no), bytes(digest)]
    for epoch, seq_no, digest in q_set:
        out += [uint64_to_bytes(epoch), uint64_to_bytes(seq_no), bytes(digest)]
    return out


def concat(slices: Sequence[bytes]) -> bytes:
    """A sequence of hash.Hash Writes hashes exactly the concatenation."""
    return b"".join(bytes(s) for s in slices)
