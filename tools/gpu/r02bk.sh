#!/bin/bash
# r02bk: randomised soak of every entry point against the oracle
# (tests/soak_gpu.py, all five case types), 280 s, seed 17.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02bk; mkdir -p $O
timeout -k 10 360 python -u tests/soak_gpu.py --seconds 280 --seed 17 2>&1 | tee $O/soak.txt
