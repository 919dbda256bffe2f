#!/bin/bash
# r02bg: randomised soak of every entry point against the oracle
# (tests/soak_gpu.py incl. launches of 65K-400K requests), 200 s, seed 11.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02bg; mkdir -p $O
timeout -k 10 290 python -u tests/soak_gpu.py --seconds 200 --seed 11 2>&1 | tee $O/soak.txt
