"""The C-ABI library loads and exports every symbol include/mirsha.h declares.
No compute calls (no GPU needed)."""
import ctypes
import os
import re

import numpy as np
import pytest

from mirbft_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "mirsha.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mirsha_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_expected_surface():
    syms = declared_symbols()
    for s in ("mirsha_ctx_create", "mirsha_hash_batch", "mirsha_hash_requests_then_batches",
              "mirsha_hash_batch_device", "mirsha_digest_lists_device", "mirsha_hash_batch_multi"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_table_matches_header():
    assert sorted(_lib.SIGNATURES) == declared_symbols()


def test_host_mirror_library_loads():
    host = ctypes.CDLL(_lib.HOST_LIB_PATH)
    assert hasattr(host, "mirbft_host_process")


def test_version_and_bucket_order_host_only():
    lib = _lib.load()
    assert lib.mirsha_version() >= 1
    from mirbft_amd import bucket_order

    lens = np.array([10, 600, 10, 5000, 70, 600, 55, 56], dtype=np.uint32)
    order, ident = bucket_order(lens)
    assert not ident
    blocks = (lens.astype(np.int64) + 72) >> 6
    # longest first, stable within a bucket
    assert list(blocks[order]) == sorted(blocks, reverse=True)
    assert sorted(order.tolist()) == list(range(lens.size))
    for b in set(blocks.tolist()):
        members = [i for i in order.tolist() if blocks[i] == b]
        assert members == sorted(members)
    same, ident2 = bucket_order(np.full(9, 272, dtype=np.uint32))
    assert ident2 and same.tolist() == list(range(9))


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.MirshaUnavailable):
        _lib.load()


def test_no_gpu_context_is_an_error_not_a_fallback():
    import torch

    if torch.cuda.is_available():
        pytest.skip("has a GPU")
    from mirbft_amd import Engine, MirshaError

    with pytest.raises(MirshaError):
        Engine(0)


def test_no_gpu_multi_is_an_error_not_a_fallback():
    """The multi-device drop-in has no CPU path either: without a device the
    context set is refused, and bad device lists are refused up front."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("has a GPU")
    from mirbft_amd import MirshaError, MultiEngine

    with pytest.raises(MirshaError):
        MultiEngine([0])
    with pytest.raises(MirshaError):
        MultiEngine([])


def test_product_library_has_no_ab_kernel_forms():
    """The retired / diagnostic CU-block forms (variants 11-15, one of which
    skips its loads) are compiled only into the tools A/B build
    (tools/ab_build.sh lib, -DMIRSHA_AB_FORMS): the product library holds the
    product instantiation of sha256_msgs_cu_kernel and no other."""
    import subprocess

    out = subprocess.run(["nm", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    forms = sorted(set(re.findall(r"sha256_msgs_cu_kernelILi(\d+)E", out)))
    assert forms == ["0"], forms
