#!/bin/bash
# r05w (5): A/B MIRSHA_ASYNC_ONE_COPY_STREAM (all SDMA copies of a submission
# on xin, digests stored by the kernel into page-locked memory) vs default;
# async GPU tests with the knob on; cgo_path 3 x 15 calls each, alternated.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05w9; mkdir -p $O
MIRSHA_AB=1 MIRSHA_ASYNC_ONE_COPY_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_submit_batch.py tests/test_gpu_multi.py tests/test_c_abi.py -x -q --timeout 150 --timeout-method thread > $O/pytest_knob.log 2>&1 || { tail -30 $O/pytest_knob.log; exit 1; }
tail -1 $O/pytest_knob.log
for r in 1 2 3; do
  MIRSHA_AB=1 MIRSHA_SUBMIT_TRACE=1 timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 15 32 nt >> $O/cgo_default.json 2>> $O/trace_default.txt || exit 1
  MIRSHA_AB=1 MIRSHA_ASYNC_ONE_COPY_STREAM=1 MIRSHA_SUBMIT_TRACE=1 timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 15 32 nt >> $O/cgo_onestream.json 2>> $O/trace_onestream.txt || exit 1
done
echo done
