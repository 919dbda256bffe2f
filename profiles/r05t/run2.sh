#!/bin/bash
# r05t (2): previous build (tools/ab_old lib + cgo_path_old: metadata on xin,
# 8 MiB first chunk then 32) vs the new one (metadata on the kernel stream,
# 8 / 16 / 32 MiB), alternated 8 times.  Both removed after the run.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05t5; mkdir -p $O
for r in 1 2 3 4 5 6 7 8; do
  LD_LIBRARY_PATH=tools/ab_old timeout -k 10 120 tests/c/build/cgo_path_old 1048576 256 15 7 32 nt >> $O/cgo_old.json 2>> $O/cgo.err || exit 1
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 nt >> $O/cgo_new.json 2>> $O/cgo.err || exit 1
done
echo done
