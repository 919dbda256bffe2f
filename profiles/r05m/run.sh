#!/bin/bash
# r05m: NUMA placement probe (tools/numa_h2d), the host-path GPU tests after
# the parallel offsets scan, and two A/Bs of the chunked Go HashBatch
# (tests/c/cgo_path.c, config 2 at full size, 32 MiB chunks): packing
# workers 8 / 12 / 15, and page-locked buffers on the GPU's NUMA node
# (MIRSHA_AB=1 MIRSHA_HOST_NUMA=1) vs hipHostMalloc's default placement.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 120 tools/numa_h2d 0 > $O/numa.json 2> $O/numa.err || echo "numa probe rc $?" >> $O/notes.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_pipeline.py tests/test_gpu_multi.py tests/test_c_abi.py tests/test_gpu_dedup_async.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for t in 8 12 15; do
    timeout -k 10 120 tests/c/build/cgo_path 1048576 256 $t 7 32 >> $O/cgo_t$t.json 2>> $O/cgo.err || exit 1
  done
done
for r in 1 2 3; do
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 >> $O/cgo_default.json 2>> $O/cgo.err || exit 1
  MIRSHA_AB=1 MIRSHA_HOST_NUMA=1 timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 >> $O/cgo_numa.json 2>> $O/cgo.err || exit 1
done
echo done
