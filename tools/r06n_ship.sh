#!/bin/bash
# The shipped round-6 tree: a 300 s randomised soak, then tools/r06f_final.sh
# (pytest -m gpu, smoke, the driver's bench command, rocprof + PMC).
set -euo pipefail
OUT=gpurun_out/r06n
mkdir -p "$OUT"
timeout -k 10 420 python -u tests/soak_gpu.py --seconds 300 --seed 6 > "$OUT/soak.log" 2>&1
bash tools/r06f_final.sh r06n
echo done
