"""CPU unit test of the library's host helpers (tests/c/host_unit.cpp, built
with g++ against mirbft_amd/csrc/mirsha_host.cpp -- no HIP): the parallel
exclusive scan behind slice-call offsets, slice packing (whole and by byte
range, as the pinned staging ring is filled chunk by chunk; plain and
streaming stores, destinations with gaps), parallel_for coverage and
per-(slot, threads) packing pools.  Built twice: optimised, and
with AddressSanitizer + UndefinedBehaviorSanitizer (host code only)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build_and_run(tmp_path, name, flags, env=None):
    exe = str(tmp_path / name)
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-pthread", *flags,
                    "-I", os.path.join(ROOT, "mirbft_amd", "csrc"), "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "host_unit.cpp"),
                    os.path.join(ROOT, "mirbft_amd", "csrc", "mirsha_host.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.strip() == "host unit ok"


def test_host_helpers(tmp_path):
    _build_and_run(tmp_path, "host_unit", ["-O2"])


def test_host_helpers_sanitized(tmp_path):
    probe = subprocess.run(["g++", "-fsanitize=address,undefined", "-x", "c++", "-", "-o", str(tmp_path / "p")],
                           input="int main(){return 0;}", capture_output=True, text=True)
    if probe.returncode != 0:
        pytest.skip("g++ without ASan/UBSan runtime")
    _build_and_run(tmp_path, "host_unit_asan",
                   ["-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                    "-fno-omit-frame-pointer"],
                   # a preloaded library (some sandboxes add one) must not stop ASan at startup
                   env=dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0"))
