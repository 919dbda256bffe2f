#!/bin/bash
# r05t (3): the library with arena-submission metadata on xin (tools/ab_old,
# built from d9259dc, removed after the run) vs on the kernel stream, the same
# cgo_path binary (8 / 16 / 32 MiB chunks), alternated 8 times: the multi leg
# (two contexts on one GPU) looked bimodal (~7 or ~14 ms) after the change.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05t6; mkdir -p $O
for r in 1 2 3 4 5 6 7 8; do
  LD_LIBRARY_PATH=tools/ab_old timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 nt >> $O/cgo_metaxin.json 2>> $O/cgo.err || exit 1
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 nt >> $O/cgo_metastream.json 2>> $O/cgo.err || exit 1
done
echo done
