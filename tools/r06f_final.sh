#!/bin/bash
# Round-6 validation of the tree: full GPU suite, smoke, the driver's bench
# command, then rocprof kernel trace + PMC passes (profiles/profile.sh).
set -euo pipefail
OUT=gpurun_out/${1:-r06f}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
timeout -k 10 900 bash profiles/profile.sh "${1:-r06f}" > "$OUT/profile.log" 2>&1
echo done
