#!/bin/bash
# r05q (2): more alternations of cgo_path old/new (the lib leg is the one the
# streaming stores touch; parallel/multi are the C mirror of the Go binding
# and do not change).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05q2; mkdir -p $O
for r in 1 2 3 4 5 6 7 8; do
  LD_LIBRARY_PATH=tools/ab_old timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 >> $O/cgo_old.json 2>> $O/cgo.err || exit 1
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 >> $O/cgo_new.json 2>> $O/cgo.err || exit 1
done
echo done
