#!/bin/bash
# Constant-schedule padding block of the identity-list chains: parity, then
# a same-box A/B against the generic final block (MIRSHA_CHAIN_PAD=0).
set -euo pipefail
OUT=gpurun_out/r06j
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "uniform_lists or pipeline_device_full_size or pipeline_overlap" > "$OUT/tests.log" 2>&1
for i in 1 2 3; do
  for pad in 1 0; do
    MIRSHA_AB=1 MIRSHA_CHAIN_PAD=$pad timeout -k 10 120 python -u bench.py --steps 200 --warmup 5 --cpu-seconds 0 --no-pcie \
      --no-config3-leg --no-overlap-extra > "$OUT/pad${pad}_$i.jsonl" 2>/dev/null
  done
done
echo done
