#!/bin/bash
# N>1 rehearsal under torchrun (the driver's SCALE launcher), every rank on
# device 0, config 2; then config 5 on one GPU with the round-6 tree.
set -euo pipefail
OUT=gpurun_out/r06m
mkdir -p "$OUT"
MIRSHA_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 4 --steps 20 --warmup 5 > "$OUT/torchrun_n4.jsonl" 2> "$OUT/torchrun_n4.err"
timeout -k 10 500 python -u bench.py --config 5 --steps 3 --warmup 1 --cpu-seconds 6 > "$OUT/c5.jsonl" 2> "$OUT/c5.err"
echo done
