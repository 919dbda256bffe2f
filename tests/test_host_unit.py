"""CPU unit test of the library's host helpers (tests/c/host_unit.cpp, built
with g++ against mirbft_amd/csrc/mirsha_host.cpp -- no HIP): the parallel
exclusive scan behind slice-call offsets, slice packing (whole and by byte
range, as the pinned staging ring is filled chunk by chunk), parallel_for
coverage and per-(slot, threads) packing pools."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_helpers(tmp_path):
    exe = str(tmp_path / "host_unit")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-pthread",
                    "-I", os.path.join(ROOT, "mirbft_amd", "csrc"), "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "host_unit.cpp"),
                    os.path.join(ROOT, "mirbft_amd", "csrc", "mirsha_host.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "host unit ok"
