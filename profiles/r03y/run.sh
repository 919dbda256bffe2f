#!/bin/bash
# r03y: randomised soak of every entry point on the final round-3 kernels
# (overlapped runs at rank priorities, per-workgroup retire) for 240 s.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03y; mkdir -p $O
timeout -k 10 330 python -u tests/soak_gpu.py --seconds 240 --seed 47 > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 1; }
tail -3 $O/soak.log
