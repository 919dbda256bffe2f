"""mirbft_amd — MI355X-native engine for MirBFT's Actions.Hash hot path.

Drop-in for the hash loop of the reference Processor (processor.go:129-143):
SHA-256 request, batch, VerifyBatch, epoch-change and checkpoint digests,
bit-exact with Go crypto/sha256, returned in origin order.  All compute runs in
hand-written gfx950 HIP kernels behind the C-ABI in include/mirsha.h.
"""
from . import eventlog, hashdata, sharding
from ._lib import MirshaError, MirshaUnavailable
from .engine import (CheckpointChains, Engine, MultiEngine, SliceArrays, Ticket, bucket_order, dedup_plan, device_count,
                     hash_batch_multi)
from .processor import (ActionResults, Actions, GpuHash, HashRequest, HashResult, PendingResults, Processor,
                        ProcessorWorkPool, gpu_hasher)

__all__ = [
    "Engine",
    "CheckpointChains",
    "SliceArrays",
    "Ticket",
    "dedup_plan",
    "PendingResults",
    "MirshaError",
    "MirshaUnavailable",
    "bucket_order",
    "device_count",
    "hash_batch_multi",
    "MultiEngine",
    "eventlog",
    "hashdata",
    "sharding",
    "ActionResults",
    "Actions",
    "GpuHash",
    "HashRequest",
    "HashResult",
    "Processor",
    "ProcessorWorkPool",
    "gpu_hasher",
]
