#!/bin/bash
# r05t: arena submissions carry only request bytes on xin (metadata on the
# kernel stream) and the chunked HashBatch opens with 8 and 16 MiB chunks;
# GPU tests of the async paths, cgo_path x6, and one memory-copy trace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05t4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_submit_batch.py tests/test_gpu_multi.py tests/test_c_abi.py tests/test_gpu_soak.py tests/test_gpu_dedup_async.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3 4 5 6; do
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 nt >> $O/cgo.json 2>> $O/cgo.err || exit 1
done
cd /tmp && timeout -k 10 200 rocprofv3 --memory-copy-trace --kernel-trace --output-format csv -d $O/prof -o run -- $GRAFT_REPO_ROOT/tests/c/build/cgo_path 1048576 256 15 2 32 nt > $O/cgo_traced.json 2> $O/trace_err.txt || exit 1
echo done
