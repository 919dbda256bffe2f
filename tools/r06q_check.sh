#!/bin/bash
# bench.py after the repeat-region and config-5 CPU-prefix changes.
set -euo pipefail
OUT=gpurun_out/r06q
mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
timeout -k 10 600 python -u bench.py --config 5 --steps 3 --warmup 1 --cpu-seconds 12 > "$OUT/c5.jsonl" 2> "$OUT/c5.err"
echo done
