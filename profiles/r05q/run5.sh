#!/bin/bash
# r05q (5): chunk bounds of the Go binding's HashBatch by binary search over
# the offsets (cgo_path) vs the linear walk (cgo_path_old, removed after the
# run), both with streamed packing, alternated.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05q5; mkdir -p $O
for r in 1 2 3 4 5 6; do
  timeout -k 10 120 tests/c/build/cgo_path_old 1048576 256 15 7 32 nt >> $O/cgo_linear.json 2>> $O/cgo.err || exit 1
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 nt >> $O/cgo_bsearch.json 2>> $O/cgo.err || exit 1
done
echo done
