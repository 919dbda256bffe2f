#!/bin/bash
# Final round-6 sources: the driver's bench command, then rocprof + PMC for
# config 2 (sequential and overlapped) and config 3 (fused and sequential),
# for profiles/traffic.json under the shipped sources' key.
set -euo pipefail
OUT=gpurun_out/r06o
mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
timeout -k 10 600 bash profiles/profile.sh r06o_c2 > "$OUT/prof_c2.log" 2>&1
timeout -k 10 600 bash profiles/profile.sh r06o_c2ovl --pipeline overlap > "$OUT/prof_c2ovl.log" 2>&1
timeout -k 10 600 bash profiles/profile.sh r06o_c3 --config 3 > "$OUT/prof_c3.log" 2>&1
timeout -k 10 600 bash profiles/profile.sh r06o_c3seq --config 3 --pipeline sequential > "$OUT/prof_c3seq.log" 2>&1
echo done
