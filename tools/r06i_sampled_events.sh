#!/bin/bash
# Sampled timing events (--event-every 4, the default) vs a bare timed loop
# (--events-in-timed-loop 0) vs events on every step (--event-every 1).
set -euo pipefail
OUT=gpurun_out/r06i
mkdir -p "$OUT"
for i in 1 2 3; do
  for mode in "every4:--event-every 4" "bare:--events-in-timed-loop 0" "every1:--event-every 1"; do
    name=${mode%%:*}; args=${mode#*:}
    timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 $args --cpu-seconds 0 --no-pcie --no-config3-leg \
      > "$OUT/${name}_$i.jsonl" 2>/dev/null
  done
done
echo done
