#!/bin/bash
# r05n: arena submissions with 4 B of metadata per gapless request and a
# quarter-size first chunk; A/B of digests stored by the kernel straight into
# the page-locked digests_out (MIRSHA_AB=1 MIRSHA_ASYNC_KERNEL_STORE=1) vs a
# D2H copy; the PCIe duplex probe.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 120 tools/numa_h2d 0 > $O/pcie.json 2> $O/pcie.err || echo "probe rc $?" >> $O/notes.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_submit_batch.py tests/test_gpu_multi.py tests/test_c_abi.py tests/test_gpu_soak.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
MIRSHA_AB=1 MIRSHA_ASYNC_KERNEL_STORE=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_submit_batch.py tests/test_gpu_multi.py tests/test_c_abi.py -x -q --timeout 150 --timeout-method thread > $O/pytest_kstore.log 2>&1 || { tail -30 $O/pytest_kstore.log; exit 1; }
tail -1 $O/pytest_kstore.log
for r in 1 2 3 4; do
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 >> $O/cgo_copy.json 2>> $O/cgo.err || exit 1
  MIRSHA_AB=1 MIRSHA_ASYNC_KERNEL_STORE=1 timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 >> $O/cgo_kstore.json 2>> $O/cgo.err || exit 1
done
echo done
