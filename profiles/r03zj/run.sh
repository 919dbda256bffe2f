#!/bin/bash
# r03zj: randomised soak of every entry point on the final round-3 kernels
# (LDS-DMA fused launch, kernel source key 6122e15229c80b8c) for 600 s.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03zj; mkdir -p $O
timeout -k 10 700 python -u tests/soak_gpu.py --seconds 600 --seed 53 > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 1; }
tail -3 $O/soak.log
