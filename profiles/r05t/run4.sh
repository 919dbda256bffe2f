#!/bin/bash
# r05t (4): A/B MIRSHA_ASYNC_HOST_META (lengths read by the scan and the kernel
# from the page-locked metadata block, no metadata copy) vs the metadata copy
# behind the request bytes on xin; async GPU tests with the knob; cgo_path
# 3 x 15 calls each, alternated.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05t9; mkdir -p $O
MIRSHA_AB=1 MIRSHA_ASYNC_HOST_META=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_submit_batch.py tests/test_gpu_multi.py tests/test_c_abi.py -x -q --timeout 150 --timeout-method thread > $O/pytest_knob.log 2>&1 || { tail -30 $O/pytest_knob.log; exit 1; }
tail -1 $O/pytest_knob.log
for r in 1 2 3; do
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 15 32 nt >> $O/cgo_copy.json 2>> $O/cgo.err || exit 1
  MIRSHA_AB=1 MIRSHA_ASYNC_HOST_META=1 timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 15 32 nt >> $O/cgo_hostmeta.json 2>> $O/cgo.err || exit 1
done
echo done
