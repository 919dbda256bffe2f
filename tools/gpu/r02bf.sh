#!/bin/bash
# r02bf: repro of soak seed 7003617 (sequential plan, mixed lengths, gaps); the
# case was exported to tools/scratch/soak (git-ignored) from tests/soak_gpu.py's draws for that seed
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02bf; mkdir -p $O
timeout -k 10 120 python -u tools/scratch/soak/repro.py 2>&1 | tee $O/repro.txt
