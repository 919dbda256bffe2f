#!/bin/bash
# The round-6 bench.py on the other BASELINE configs (one GPU).
set -euo pipefail
OUT=gpurun_out/r06p
mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py --config 1 > "$OUT/c1.jsonl" 2> "$OUT/c1.err"
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 6 > "$OUT/c3.jsonl" 2> "$OUT/c3.err"
timeout -k 10 300 python -u bench.py --config 4 --steps 20 --warmup 5 --cpu-seconds 6 > "$OUT/c4.jsonl" 2> "$OUT/c4.err"
echo done
