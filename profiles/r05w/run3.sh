#!/bin/bash
# r05w (3): exact-fit buffer growth (tools/ab_old, the library before the
# headroom fix, removed after the run) vs 1.5x headroom, same cgo_path binary,
# alternated 3 x 15 calls; per call: ms, longest worker wait, longest submit.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05w4; mkdir -p $O
for r in 1 2 3; do
  LD_LIBRARY_PATH=tools/ab_old timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 15 32 nt >> $O/cgo_exact.json 2>> $O/cgo.err || exit 1
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 15 32 nt >> $O/cgo_headroom.json 2>> $O/cgo.err || exit 1
done
echo done
