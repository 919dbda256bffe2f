#!/bin/bash
# r05s (3): ring of 4 staging slots (4 chunks queued before the plan) vs 3.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05s3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_pipeline.py tests/test_c_abi.py tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  MIRSHA_AB=1 MIRSHA_AB_LIB=tools/ab_old/libmirsha.so timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --cpu-seconds 0 >> $O/bench_old.jsonl 2>> $O/bench.err || exit 1
  timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --cpu-seconds 0 >> $O/bench_new.jsonl 2>> $O/bench.err || exit 1
done
MIRSHA_AB=1 MIRSHA_STAGE_TRACE=1 timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --cpu-seconds 0 > $O/bench_trace.jsonl 2> $O/trace_after.txt || exit 1
echo done
