#!/bin/bash
# Final shipped-tree check after the event_steps refactor: smoke, GPU suite, default bench line.
set -euo pipefail
OUT=gpurun_out/r06r
mkdir -p "$OUT"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
timeout -k 10 300 python -u bench.py > "$OUT/bench_default.jsonl" 2> "$OUT/bench_default.err"
echo done
