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


def epoch_change_payload(new_epoch: int, origin: int, n_checkpoints: int, n_p: int, n_q: int,
                         seed: int = 0) -> list[bytes]:
    """One origin's EpochChange as epochChangeHashData slices (stateless.go:311-340),
    with deterministic synthetic checkpoint values / P / Q digests.  Sequence
    numbers follow persisted.constructEpochChange (persisted.go:244-317): C
    checkpoints one interval apart, then one P and one Q entry per sequence."""
    import numpy as np

    rng = np.random.default_rng([seed, origin, new_epoch])
    vals = rng.integers(0, 256, size=(n_checkpoints + n_p + n_q, 32), dtype=np.uint8)
    cps = [((k + 1) * 320, vals[k].tobytes()) for k in range(n_checkpoints)]
    base = n_checkpoints * 320
    p_set = [(new_epoch - 1, base + k + 1, vals[n_checkpoints + k].tobytes()) for k in range(n_p)]
    q_set = [(new_epoch - 1, base + k + 1, vals[n_checkpoints + n_p + k].tobytes()) for k in range(n_q)]
    return epoch_change_hash_data(new_epoch, cps, p_set, q_set)


def epoch_change_cycle(n_nodes: int, n_requests: int, n_checkpoints: int, n_p: int, n_q: int,
                       new_epoch: int = 2, seed: int = 0):
    """One node's Ready() cycle during an epoch change (BASELINE config 4 stand-in):
    request r is the EpochChangeAck hash of origin r % n_nodes as relayed by
    source r // n_nodes (applyEpochChangeAckMsg, epoch_target.go:459-477), so
    every origin's payload recurs once per source.  Each request gets its OWN
    copy of the bytes (acks are deserialized separately), laid out as slices
    of one buffer.  Returns (buf, slice_off, slice_len, first, origin)."""
    import numpy as np

    payloads = [concat(epoch_change_payload(new_epoch, o, n_checkpoints, n_p, n_q, seed)) for o in range(n_nodes)]
    pattern = np.array([8] + [8, 32] * n_checkpoints + [8, 8, 32] * (n_p + n_q), dtype=np.uint64)
    plen = int(pattern.sum())
    origin = (np.arange(n_requests) % n_nodes).astype(np.int64)
    buf = np.frombuffer(b"".join(payloads), dtype=np.uint8).reshape(n_nodes, plen)[origin].reshape(-1).copy()
    rel = np.zeros(pattern.size, dtype=np.uint64)
    np.cumsum(pattern[:-1], out=rel[1:])
    slice_off = (np.arange(n_requests, dtype=np.uint64)[:, None] * np.uint64(plen) + rel[None, :]).reshape(-1)
    slice_len = np.tile(pattern, n_requests)
    first = (np.arange(n_requests + 1, dtype=np.int64) * pattern.size).astype(np.uint32)
    return buf, slice_off, slice_len, first, origin
