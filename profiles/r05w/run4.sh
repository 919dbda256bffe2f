#!/bin/bash
# r05w (4): where do the ~9 ms blocking hipMemcpyAsync calls inside
# mirsha_submit_batch come from?  cgo_path (2 x 15 calls) under the default
# runtime, with 8 hardware queues, and with SDMA off (blit-kernel copies);
# MIRSHA_SUBMIT_TRACE prints each submit slower than 2 ms.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05w8; mkdir -p $O
for v in default hwq8 nosdma; do
  case $v in
    default) E="";;
    hwq8) E="GPU_MAX_HW_QUEUES=8";;
    nosdma) E="HSA_ENABLE_SDMA=0";;
  esac
  for r in 1 2; do
    env $E MIRSHA_AB=1 MIRSHA_SUBMIT_TRACE=1 timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 15 32 nt >> $O/cgo_$v.json 2>> $O/trace_$v.txt || exit 1
  done
done
echo done
