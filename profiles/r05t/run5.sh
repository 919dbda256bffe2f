#!/bin/bash
# r05t (5): the synchronous slice call reuses its host scratch (lengths,
# packed offsets) and validates without an n-sized error array: slice GPU
# tests, then cgo_path's `lib` leg (mirsha_hash_slices) old (tools/ab_old,
# removed after the run) vs new, alternated.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05t11; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dedup_async.py tests/test_gpu_host_pipeline.py tests/test_c_abi.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3 4; do
  LD_LIBRARY_PATH=tools/ab_old timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 9 32 nt >> $O/cgo_old.json 2>> $O/cgo.err || exit 1
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 9 32 nt >> $O/cgo_new.json 2>> $O/cgo.err || exit 1
done
echo done
