"""Host-side mirror of the reference's Processor hash path (Python binding).

reference (Go, github.com/IBM/mirbft)              here
------------------------------------------------  -------------------------------------
type Hasher func() hash.Hash      processor.go:21  ``Hasher`` = callable returning ``GpuHash``
HashRequest{Data, Origin}   actions.go:157-164     ``HashRequest(data, origin)``
HashResult{Digest, Request} actions.go:224-230     ``HashResult(digest, request)``
ActionResults{Digests, Checkpoints} :218-221       ``ActionResults``
(*Processor).Process        processor.go:65-171    ``Processor.process`` (hash loop :129-143)
ProcessorWorkPool.Process   processor.go:447-470   ``ProcessorWorkPool.process``

``Processor.process`` coalesces every HashRequest of one Ready() cycle into a
single batched device call and returns ``Digests[i]`` for ``actions.hash[i]``
with the request back-pointer (origin order).  The reference's work pool
returns digests in completion order (processor.go:349-356); this one keeps
origin order, which is a legal (and deterministic) completion order.
Failures raise (the reference panics, processor.go:75,81,85,91).

``dedup=True`` hashes each distinct request content once per cycle and hands
every duplicate its own digest (epoch-change acks: applyEpochChangeAckMsg,
epoch_target.go:459-477).  ``Processor.submit`` / ``PendingResults.wait`` is
the asynchronous form (mirsha_submit_slices / mirsha_wait): the cycle's
requests are packed before ``submit`` returns and the digests are collected,
in origin order, after the caller's other work for the cycle.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import Any, Callable, Optional

from .engine import Engine


@dataclass(eq=False)
class HashRequest:
    data: list  # [][]byte; concatenation is hashed
    origin: Any = None  # opaque to the hasher (actions.go:152-156)


@dataclass(eq=False)
class HashResult:
    digest: bytes
    request: HashRequest


@dataclass(eq=False)
class Actions:
    """Subset of mirbft.Actions (actions.go:18-52) the hash path reads."""

    hash: list = field(default_factory=list)


@dataclass(eq=False)
class ActionResults:
    digests: list = field(default_factory=list)
    checkpoints: list = field(default_factory=list)


class GpuHash:
    """hash.Hash (Write / Sum / Reset / Size / BlockSize) whose Sum runs on the GPU."""

    size = 32
    block_size = 64

    def __init__(self, engine: Engine):
        self._engine = engine
        self._parts: list[bytes] = []

    def write(self, data: bytes) -> int:
        self._parts.append(bytes(data))
        return len(data)

    def sum(self, b: bytes = b"") -> bytes:
        return bytes(b) + self._engine.hash_slices([self._parts])[0].tobytes()

    def reset(self) -> None:
        self._parts = []


def gpu_hasher(engine: Engine) -> Callable[[], GpuHash]:
    """A `Hasher` factory (processor.go:21) backed by the GPU."""
    return lambda: GpuHash(engine)


def _results(reqs, digests) -> ActionResults:
    results = ActionResults(digests=[None] * len(reqs))
    for i, req in enumerate(reqs):  # Digests[i] for actions.Hash[i] (processor.go:139)
        results.digests[i] = HashResult(digest=digests[i].tobytes(), request=req)
    return results


class PendingResults:
    """Hash results of one submitted cycle; ``wait()`` returns its ActionResults."""

    def __init__(self, engine: Engine, reqs, ticket):
        self._engine, self._reqs, self._ticket = engine, reqs, ticket
        self._results: Optional[ActionResults] = None

    def done(self) -> bool:
        return self._results is not None or self._ticket is None or self._engine.poll(self._ticket)

    def wait(self) -> ActionResults:
        if self._results is None:
            digests = self._engine.wait(self._ticket) if self._ticket is not None else []
            self._results = _results(self._reqs, digests)
        return self._results


class Processor:
    """Hash stage of mirbft.Processor; batches one Ready() cycle per device call."""

    def __init__(self, engine: Optional[Engine] = None, device: int = 0, dedup: bool = False):
        self.engine = engine if engine is not None else Engine(device)
        self.dedup = dedup

    def process(self, actions: Actions) -> ActionResults:
        reqs = actions.hash
        if not reqs:
            return ActionResults(digests=[])
        return _results(reqs, self.engine.hash_slices([r.data for r in reqs], dedup=self.dedup))

    def submit(self, actions: Actions) -> PendingResults:
        """Asynchronous process(): queue the cycle's hashing, return at once."""
        reqs = list(actions.hash)
        ticket = self.engine.submit_slices([r.data for r in reqs], dedup=self.dedup) if reqs else None
        return PendingResults(self.engine, reqs, ticket)


class ProcessorWorkPool(Processor):
    """ProcessorWorkPool (processor.go:183-197): serialised Process, batched hashing.

    ``hash_workers`` is accepted for API parity (processor.go:396-399); the device
    replaces the goroutine pool.
    """

    def __init__(self, engine: Optional[Engine] = None, device: int = 0, hash_workers: int = 0,
                 transmit_workers: int = 0, dedup: bool = False):
        super().__init__(engine, device, dedup)
        self._mutex = threading.Lock()
        self.hash_workers = hash_workers

    def process(self, actions: Actions, overlap: Optional[Callable[[], Any]] = None) -> ActionResults:
        """processor.go:447-470: the pool hashes while the WAL and the sends
        proceed.  Here the cycle's hashing is submitted first, ``overlap()``
        (the caller's persist / transmit work) runs while the GPU hashes, then
        the digests are collected in origin order."""
        with self._mutex:  # processor.go:448-449
            pending = self.submit(actions)
            if overlap is not None:
                overlap()
            return pending.wait()

    def stop(self) -> None:
        pass
