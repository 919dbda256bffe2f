#!/bin/bash
# r05q: non-temporal (streaming) stores when the library packs into its
# page-locked DMA staging (the ring's fill, arena/slice submissions).  A/B
# against the previous build (tools/ab_old/libmirsha.so, plain stores):
# cgo_path's `lib` leg (mirsha_hash_slices packing into the ring) and the
# bench's pcie_inclusive (pageable arena copied into the ring), alternated
# on one box.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  LD_LIBRARY_PATH=tools/ab_old timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 >> $O/cgo_old.json 2>> $O/cgo.err || exit 1
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 >> $O/cgo_new.json 2>> $O/cgo.err || exit 1
done
for r in 1 2; do
  MIRSHA_AB=1 MIRSHA_AB_LIB=tools/ab_old/libmirsha.so timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 >> $O/bench_old.jsonl 2>> $O/bench.err || exit 1
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 >> $O/bench_new.jsonl 2>> $O/bench.err || exit 1
done
echo done
