#!/bin/bash
# r02bh: randomised soak of every entry point against the oracle
# (tests/soak_gpu.py with checkpoint-chain cases), 200 s, seed 13.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02bh; mkdir -p $O
timeout -k 10 290 python -u tests/soak_gpu.py --seconds 200 --seed 13 2>&1 | tee $O/soak.txt
