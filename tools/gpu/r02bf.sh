#!/bin/bash
# r02bf: repro of soak seed 7003617 (sequential plan, mixed lengths, gaps)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02bf; mkdir -p $O
timeout -k 10 120 python -u tools/scratch/soak/repro.py 2>&1 | tee $O/repro.txt
