#!/bin/bash
# r05w (6): single-copy-stream arena submissions as the default: the whole
# GPU suite, then cgo_path 3 x 15 calls and the default bench line.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05w10; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2 3; do
  MIRSHA_AB=1 MIRSHA_SUBMIT_TRACE=1 timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 15 32 nt >> $O/cgo.json 2>> $O/trace.txt || exit 1
done
timeout -k 10 300 python -u bench.py > $O/bench.jsonl 2> $O/bench.err || exit 1
echo done
