#!/bin/bash
# r02be: randomised soak of every entry point against the oracle
# (tests/soak_gpu.py), 150 s.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02be; mkdir -p $O
timeout -k 10 240 python -u tests/soak_gpu.py --seconds 150 --seed 7 2>&1 | tee $O/soak.txt
