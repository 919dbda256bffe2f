#!/bin/bash
# r05q (3): the C mirror of the Go binding packing with non-temporal stores
# (cgo_path ... nt) vs plain stores, alternated on one box; test_c_abi on GPU.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05q3; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_c_abi.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3 4 5 6 7 8; do
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 plain >> $O/cgo_plain.json 2>> $O/cgo.err || exit 1
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 nt >> $O/cgo_nt.json 2>> $O/cgo.err || exit 1
done
echo done
