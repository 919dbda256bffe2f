#!/bin/bash
# r05w (2): grow-only buffers with 1.5x headroom (the exact-fit growth freed
# and reallocated ring-slot buffers now and then: hipFree drains the device,
# a ~9 ms submit).  Host-path GPU tests, then cgo_path 3 x 15 calls with the
# per-call longest submit.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05w3; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_submit_batch.py tests/test_gpu_multi.py tests/test_c_abi.py tests/test_gpu_soak.py tests/test_gpu_dedup_async.py tests/test_gpu_host_pipeline.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 15 32 nt >> $O/cgo.json 2>> $O/cgo.err || exit 1
done
echo done
