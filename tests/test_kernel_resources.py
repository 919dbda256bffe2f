"""Register budget of the product kernels (CPU: hipcc's resource-usage remarks
for gfx950, device code only, ~5 s).  A kernel that spills to scratch or
drops below its occupancy runs measurably slower (the fused
launch once grew 48 B per lane of scratch from one inlined helper, +70 us on
config 3, profiles/r02az), and nothing else in the CPU suite would notice."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mirbft_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

# kernel (demangled-name substring) -> minimum waves per SIMD
OCCUPANCY = {
    "sha256_msgs_kernelILb1ELb0E": 8,      # the request kernel (LDS loader, 32-bit buffers)
    "sha256_msgs_kernelILb1ELb1E": 6,      # > 4 GiB arenas (64-bit addressing)
    "sha256_msgs_overlap_kernel": 8,       # overlapped cycles
    "sha256_fused_paced_kernel": 4,        # fused config-3 launch (4 tile waves per SIMD)
    "sha256_msgs_cu_kernel": 4,            # CU-block request kernel (4 waves per SIMD, prefetching)
    "sha256_chain_kernel": 8,
}


@pytest.fixture(scope="module")
def resources(tmp_path_factory):
    if not os.path.exists(HIPCC) and not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("res") / "k.o"
    r = subprocess.run([HIPCC if os.path.exists(HIPCC) else "hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "--cuda-device-only", "-c", "mirsha_kernels.hip", "-o", str(out),
                        "-Rpass-analysis=kernel-resource-usage"],
                       cwd=CSRC, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    kernels, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = kernels.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+) \[-Rpass", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    assert kernels, r.stderr[-2000:]
    return kernels


def test_no_scratch_or_spills(resources):
    bad = {k: v for k, v in resources.items()
           if v.get("ScratchSize", 0) or v.get("VGPRs Spill", 0)}
    assert not bad, f"kernels spilling to scratch: {bad}"


@pytest.mark.parametrize("name,occ", sorted(OCCUPANCY.items()))
def test_occupancy(resources, name, occ):
    hits = {k: v for k, v in resources.items() if name in k}
    assert hits, f"{name} not compiled"
    for k, v in hits.items():
        assert v.get("Occupancy", 0) >= occ, f"{k}: {v}"
