#!/bin/bash
# r04j: the multi-device tests (now with four contexts) and a 300 s
# randomised soak over every entry point on the round-4 head.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04j; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -v --timeout 120 --timeout-method thread > $O/pytest_multi.log 2>&1 || { tail -40 $O/pytest_multi.log; exit 1; }
tail -1 $O/pytest_multi.log
timeout -k 10 400 python -u tests/soak_gpu.py --seconds 300 --seed 97 > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 1; }
tail -2 $O/soak.log
echo all done
