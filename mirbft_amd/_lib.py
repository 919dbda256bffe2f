"""ctypes binding of the C-ABI in include/mirsha.h (the product's only native boundary).

The shared library is built in-tree (``mirbft_amd/lib/libmirsha.so``) by
``__graft_entry__.build()``.  There is NO fallback: if the library is missing,
loading fails loudly, and every compute call goes through the HIP kernels.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_uint8, c_uint32, c_uint64, c_void_p

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.path.join(LIB_DIR, "libmirsha.so")
HOST_LIB_PATH = os.path.join(LIB_DIR, "libmirbft_host.so")

MIRSHA_OK = 0
MIRSHA_EINVAL = -1
MIRSHA_EHIP = -2
MIRSHA_ENOMEM = -3
MIRSHA_ERANGE = -4
MIRSHA_ENODEV = -5
MIRSHA_NULL_INDEX = 0xFFFFFFFF
MIRSHA_MAX_MESSAGE_BYTES = 0xFFFFFF00
MIRSHA_MAX_DEVICE_ARENA_BYTES = 0xFFFFFF00
MIRSHA_SUBMIT_DEDUP = 1

ERROR_NAMES = {
    MIRSHA_EINVAL: "EINVAL",
    MIRSHA_EHIP: "EHIP",
    MIRSHA_ENOMEM: "ENOMEM",
    MIRSHA_ERANGE: "ERANGE",
    MIRSHA_ENODEV: "ENODEV",
}

# Every symbol include/mirsha.h declares, with (restype, argtypes).
_u8p = POINTER(c_uint8)
_u32p = POINTER(c_uint32)
_u64p = POINTER(c_uint64)
SIGNATURES = {
    "mirsha_version": (c_int, []),
    "mirsha_device_count": (c_int, [POINTER(c_int)]),
    "mirsha_ctx_create": (c_int, [c_int, POINTER(c_void_p)]),
    "mirsha_ctx_destroy": (None, [c_void_p]),
    "mirsha_last_error": (c_char_p, [c_void_p]),
    "mirsha_ctx_set_stream": (c_int, [c_void_p, c_void_p]),
    "mirsha_ctx_stream": (c_void_p, [c_void_p]),
    "mirsha_ctx_set_variant": (c_int, [c_void_p, c_int]),
    "mirsha_ctx_set_timing": (c_int, [c_void_p, c_int]),
    "mirsha_ctx_set_timing_mask": (c_int, [c_void_p, c_uint32]),
    "mirsha_ctx_kernel_time": (c_int, [c_void_p, c_int, _u64p, POINTER(c_double)]),
    "mirsha_ctx_reset_timing": (c_int, [c_void_p]),
    "mirsha_sync": (c_int, [c_void_p]),
    "mirsha_hash_batch": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_uint32, c_void_p]),
    "mirsha_hash_slices": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_void_p]),
    "mirsha_hash_slices_dedup": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_void_p, _u32p]),
    "mirsha_dedup_plan": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p, _u32p]),
    "mirsha_host_alloc": (c_int, [c_void_p, c_uint64, POINTER(c_void_p)]),
    "mirsha_host_free": (None, [c_void_p]),
    "mirsha_submit_slices": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_void_p, c_int, _u64p]),
    "mirsha_wait": (c_int, [c_void_p, c_uint64]),
    "mirsha_poll": (c_int, [c_void_p, c_uint64, POINTER(c_int)]),
    "mirsha_submit_batch": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_uint32, c_void_p, _u64p]),
    "mirsha_hash_requests_then_batches": (
        c_int,
        [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_uint32, c_void_p, c_void_p],
    ),
    "mirsha_digest_lists": (c_int, [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_uint32, c_void_p]),
    "mirsha_hash_batch_device": (
        c_int,
        [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_uint32, c_void_p],
    ),
    "mirsha_digest_lists_device": (
        c_int,
        [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_uint32, c_uint32, c_void_p],
    ),
    "mirsha_bucket_order": (c_int, [c_void_p, c_uint32, c_void_p]),
    "mirsha_pipeline_create": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_uint32, POINTER(c_void_p)]),
    "mirsha_pipeline_create_mode": (
        c_int,
        [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_uint32, c_int, POINTER(c_void_p)],
    ),
    "mirsha_pipeline_destroy": (None, [c_void_p]),
    "mirsha_pipeline_mode": (c_int, [c_void_p]),
    "mirsha_pipeline_fallback": (c_int, [c_void_p]),
    "mirsha_pipeline_status": (c_int, [c_void_p, c_void_p]),
    "mirsha_pipeline_trace": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, POINTER(c_uint64)]),
    "mirsha_pipeline_shape": (c_int, [c_void_p, _u32p, _u32p, _u32p]),
    "mirsha_pipeline_split_tiles": (c_int, [c_void_p, _u32p, _u32p]),
    "mirsha_pipeline_segments": (c_int, [c_void_p, _u32p, _u32p, c_uint32]),
    "mirsha_hash_requests_then_batches_device": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "mirsha_pipeline_overlap_device": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "mirsha_chains_create": (c_int, [c_void_p, c_uint32, POINTER(c_void_p)]),
    "mirsha_chains_destroy": (None, [c_void_p]),
    "mirsha_chains_absorb": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint32]),
    "mirsha_chains_sum": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p]),
    "mirsha_chains_reset": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32]),
    "mirsha_hash_batch_multi": (
        c_int,
        [c_void_p, c_int, c_void_p, c_uint64, c_void_p, c_void_p, c_uint32, c_void_p],
    ),
    "mirsha_multi_release": (None, []),
    "mirsha_multi_create": (c_int, [c_void_p, c_int, POINTER(c_void_p)]),
    "mirsha_multi_destroy": (None, [c_void_p]),
    "mirsha_multi_last_error": (c_char_p, [c_void_p]),
    "mirsha_multi_devices": (c_int, [c_void_p]),
    "mirsha_multi_ctx": (c_void_p, [c_void_p, c_int]),
    "mirsha_multi_last_cut": (c_int, [c_void_p, _u32p, c_int]),
    "mirsha_hash_slices_multi": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_void_p]),
    "mirsha_submit_slices_multi": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_void_p, c_int, _u64p],
    ),
    "mirsha_hash_arena_multi": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_uint32, c_void_p]),
    "mirsha_multi_host_alloc": (c_int, [c_void_p, c_uint64, POINTER(c_void_p)]),
    "mirsha_submit_arena_multi": (
        c_int,
        [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_uint32, c_void_p, _u64p],
    ),
    "mirsha_wait_multi": (c_int, [c_void_p, c_uint64]),
    "mirsha_poll_multi": (c_int, [c_void_p, c_uint64, POINTER(c_int)]),
    "mirsha_multi_host_profile": (c_int, [c_void_p, c_int, POINTER(c_double), c_int]),
    "mirsha_synth_requests_device": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_uint32, c_void_p]),
    "mirsha_synth_mixed_lengths_device": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_void_p]),
    "mirsha_synth_mixed_device": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_void_p, c_void_p]),
    "mirsha_clock_probe": (c_int, [c_void_p, c_uint32, POINTER(c_double), POINTER(c_double)]),
    "mirsha_ctx_host_profile": (c_int, [c_void_p, POINTER(c_double), c_int]),
}


class MirshaUnavailable(RuntimeError):
    """The HIP library is not built / cannot be loaded.  Never silently bypassed."""


class MirshaError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"mirsha error {code} ({ERROR_NAMES.get(code, '?')}): {message}")
        self.code = code


_lib = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    # MIRSHA_AB_LIB: an A/B build of the same sources (tools/ab_build.sh) for
    # same-box timing comparisons; never set by tests, smoke() or the driver.
    path = os.environ.get("MIRSHA_AB_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise MirshaUnavailable(
            f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950).  There is no CPU fallback."
        )
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        if os.environ.get("MIRSHA_AB_LIB") and not hasattr(lib, name):
            continue  # an older A/B build: symbols added since are absent
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, ctx=None) -> None:
    if rc != MIRSHA_OK:
        msg = ""
        if ctx is not None:
            raw = load().mirsha_last_error(ctx)
            msg = raw.decode() if raw else ""
        raise MirshaError(rc, msg)
