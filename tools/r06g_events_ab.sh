#!/bin/bash
# Does recording HIP events around the request kernel inside the timed loop
# lengthen the measured step?  Same box, alternated.
set -euo pipefail
OUT=gpurun_out/r06g
mkdir -p "$OUT"
for i in 1 2 3; do
  for ev in 1 0; do
    for st in 20 200; do
      timeout -k 10 120 python -u bench.py --steps $st --warmup 5 --events-in-timed-loop $ev --cpu-seconds 0 --no-pcie \
        --no-config3-leg --no-overlap-extra > "$OUT/ev${ev}_s${st}_$i.jsonl" 2>/dev/null
    done
  done
done
echo done
