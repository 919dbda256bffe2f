#!/bin/bash
# Timing events bound to the kernel dispatch (hipExtLaunchKernel) instead of
# hipEventRecord markers: does the timed loop still lengthen with events on,
# and do the event durations agree with rocprof?  Same box.
set -euo pipefail
OUT=gpurun_out/r06h
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "timing or kernel_time or clock or pipeline_device_full_size or uniform" > "$OUT/tests.log" 2>&1
for i in 1 2 3; do
  for ev in 1 0; do
    timeout -k 10 120 python -u bench.py --steps 200 --warmup 5 --events-in-timed-loop $ev --cpu-seconds 0 --no-pcie \
      --no-config3-leg > "$OUT/ev${ev}_$i.jsonl" 2>/dev/null
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-config3-leg > "$OUT/bench_under_trace.jsonl" 2> "$OUT/trace.err"
echo done
