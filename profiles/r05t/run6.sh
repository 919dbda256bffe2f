#!/bin/bash
# r05t (6): the chunked HashBatch with the offsets pass folded into the
# packing (one lengths pass by blocks, offsets written per block by the
# packing workers) vs the two-pass offsets (cgo_path_old, removed after the
# run): the C-ABI GPU tests, then 4 pairs alternated.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05t13; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_c_abi.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3 4; do
  timeout -k 10 120 tests/c/build/cgo_path_old 1048576 256 15 9 32 nt >> $O/cgo_twopass.json 2>> $O/cgo.err || exit 1
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 9 32 nt >> $O/cgo_folded.json 2>> $O/cgo.err || exit 1
done
echo done
